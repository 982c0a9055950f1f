#!/bin/bash
# Round-6 session h4: the dispatch-chunk threshold at the per-rank set sizes of N = 2 and N = 4 (32 and 16 views):
# FIN = the in-tree final build (small chunks for sets of >= 32 views), BIG65 = never (chunk 8 throughout, as before
# item 34), BIG16 = small chunks from 16 views on; alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
FIN=$PWD/threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so
run() {  # name lib tag args...
  local name=$1 lib=$2 tag=$3; shift 3
  GSR_HIP_LIB=$lib timeout -k 10 300 python -u bench.py $BASE "$@" \
    > gpurun_out/r06h4_${tag}_${name}.json 2> gpurun_out/r06h4_${tag}_${name}.log || exit 1
  python scripts/bench_summary.py gpurun_out/r06h4_${tag}_${name}.json
}
for round in 1 2; do
  run FIN $FIN v32_$round --views 32 --steps 20 --warmup 3
  run BIG65 $PWD/build_ab/libgsr_hip_BIG65.so v32_$round --views 32 --steps 20 --warmup 3
  run FIN $FIN v16_$round --views 16 --steps 20 --warmup 3
  run BIG16 $PWD/build_ab/libgsr_hip_BIG16.so v16_$round --views 16 --steps 20 --warmup 3
done
echo "r06h4 done"
