#!/bin/bash
# Round-6 session z6: B0 (HEAD: dispatch-order chunk 8 for every blend launch) vs NEW (the in-tree library: chunk 2
# for the forwards and 4 for the backwards of sets of 32 views or more, 8 below; order_chunk), headline / C5
# alternated, 8-view sets once; then the whole -m gpu suite on NEW.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
run() {  # name lib tag args...
  local name=$1 lib=$2 tag=$3; shift 3
  GSR_HIP_LIB=$lib timeout -k 10 300 python -u bench.py $BASE "$@" \
    > gpurun_out/r06z6_${tag}_${name}.json 2> gpurun_out/r06z6_${tag}_${name}.log || exit 1
  python scripts/bench_summary.py gpurun_out/r06z6_${tag}_${name}.json
}
NEW=$PWD/threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so
for round in 1 2; do
  run B0 $PWD/build_ab/libgsr_hip_B0.so v64_$round --steps 10 --warmup 3
  run NEW $NEW v64_$round --steps 10 --warmup 3
  run B0 $PWD/build_ab/libgsr_hip_B0.so c5_$round --workload sugar --steps 10 --warmup 3
  run NEW $NEW c5_$round --workload sugar --steps 10 --warmup 3
done
run B0 $PWD/build_ab/libgsr_hip_B0.so v8 --views 8 --steps 30 --warmup 5
run NEW $NEW v8 --views 8 --steps 30 --warmup 5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06z6_gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06z6_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06z6_gpu_tests.log
echo "r06z6 done"
