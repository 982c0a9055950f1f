#!/bin/bash
# Round-6 session f: M vs N (partial-group replay without dead reads, no recompute-cull path) on the headline and
# the 8-view set, then the whole -m gpu suite on the in-tree library (N).
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in M=build_ab/libgsr_hip_M.so N=build_ab/libgsr_hip_N.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06f_${tag}_${name}_${round}.json \
        2> gpurun_out/r06f_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06f_${tag}_${name}_${round}.json
    done
  done
done
T=r06f STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
