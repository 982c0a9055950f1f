#!/bin/bash
# Round-6 session t: B0 (HEAD) vs W7 (the one-colour tile forward at 7 waves per SIMD: 72 VGPRs, one spilled outside the loop) vs VG5 (the one-colour k_view_grad at 5 waves per SIMD: 95 VGPRs, 3 spilled, reloaded per item before its means2D store),
# headline and 8-view sets alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in B0=build_ab/libgsr_hip_B0.so W7=build_ab/libgsr_hip_W7.so VG5=build_ab/libgsr_hip_VG5.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06t_${tag}_${name}_${round}.json \
        2> gpurun_out/r06t_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06t_${tag}_${name}_${round}.json
    done
  done
done
echo "r06t ab done"
echo "r06t done"
