#!/bin/bash
# Round-6 session z3: the blends' dispatch-order chunk (GSR_ORDER_CHUNK: views whose super-tiles are ordered
# heaviest-first together; tuned in round 2 at 4 = 8) re-swept on the final kernels: 2 / 4 / 8 (HEAD) / 16,
# headline alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for name in CH8 CH2 CH4 CH16; do
    GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u bench.py $BASE --steps 10 --warmup 3 \
      > gpurun_out/r06z3_v64_${name}_${round}.json 2> gpurun_out/r06z3_v64_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06z3_v64_${name}_${round}.json
  done
done
echo "r06z3 done"
