#!/bin/bash
# Round-6 session u: B0 (HEAD) vs S7 (the keys-only LDS-atomic-rank tile-sort scatter at 7 waves per SIMD: 72 VGPRs, 4 spilled; the LDS allows 7 workgroups per CU),
# headline and C5 alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in B0=build_ab/libgsr_hip_B0.so S7=build_ab/libgsr_hip_S7.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "c5:--workload sugar --steps 10 --warmup 3"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06u_${tag}_${name}_${round}.json \
        2> gpurun_out/r06u_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06u_${tag}_${name}_${round}.json
    done
  done
done
echo "r06u ab done"
echo "r06u done"
