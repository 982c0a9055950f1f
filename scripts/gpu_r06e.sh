#!/bin/bash
# Round-6 session e: small-set and per-view lines, L (HEAD) vs M (quadrant-wave forward loop trims), and the
# tile-wave forward forced for 8-view sets; each run under its own time limit, the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in L=build_ab/libgsr_hip_L.so M=build_ab/libgsr_hip_M.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v8:--views 8 --steps 30 --warmup 5" "pv:--path per-view --views 16 --steps 3 --warmup 1" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06e_${tag}_${name}_${round}.json \
        2> gpurun_out/r06e_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06e_${tag}_${name}_${round}.json
    done
    GSR_FWD_KERNEL=tile GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE --views 8 --steps 30 --warmup 5 \
      > gpurun_out/r06e_v8tile_${name}_${round}.json 2> gpurun_out/r06e_v8tile_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06e_v8tile_${name}_${round}.json
  done
done
echo "r06e done"
