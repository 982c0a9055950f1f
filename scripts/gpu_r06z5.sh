#!/bin/bash
# Round-6 session z5: the dispatch-order chunk split between the forward blends (GSR_ORDER_CHUNK_FWD) and the
# backward blends (GSR_ORDER_CHUNK); F<f>B<b> = forward chunk f, backward chunk b (HEAD: F8B8). Session z3 found the
# forward 11 % faster at chunk 2 with the backward slightly slower. Headline and C5 alternated, then 8-view sets.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
run() {  # name tag args...
  local name=$1 tag=$2; shift 2
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u bench.py $BASE "$@" \
    > gpurun_out/r06z5_${tag}_${name}.json 2> gpurun_out/r06z5_${tag}_${name}.log || exit 1
  python scripts/bench_summary.py gpurun_out/r06z5_${tag}_${name}.json
}
for round in 1 2; do
  for name in F8B8 F2B8 F1B8 F2B4; do
    run $name v64_$round --steps 10 --warmup 3
    run $name c5_$round --workload sugar --steps 10 --warmup 3
  done
done
for name in F8B8 F2B8 F1B8; do run $name v8 --views 8 --steps 30 --warmup 5; done
echo "r06z5 done"
