#!/bin/bash
# Round-6 session h: O (HEAD) vs P (both forwards keep the next-next index raw until the next batch and store the
# cull bytes after the next loads) on the headline, the 8-view set and C5, then the whole -m gpu suite on P.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in O=build_ab/libgsr_hip_O.so P=build_ab/libgsr_hip_P.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06h_${tag}_${name}_${round}.json \
        2> gpurun_out/r06h_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06h_${tag}_${name}_${round}.json
    done
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_P.so T=r06h STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
