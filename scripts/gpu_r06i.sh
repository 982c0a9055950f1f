#!/bin/bash
# Round-6 session i: Q (the sort scatter's in-wave ranks from LDS atomic adds with return instead of ballot digit
# matching; stable only if a wave's same-address LDS atomics are serviced in lane order) — the GPU sort tests on Q
# first, then P (HEAD) vs Q on the headline, the 8-view set and C5, then the whole gpu suite on Q.
set -o pipefail
mkdir -p gpurun_out
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_Q.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r06i_sort_Q.log 2>&1 || { tail -30 gpurun_out/r06i_sort_Q.log; exit 1; }
tail -2 gpurun_out/r06i_sort_Q.log
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in P=build_ab/libgsr_hip_P.so Q=build_ab/libgsr_hip_Q.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06i_${tag}_${name}_${round}.json \
        2> gpurun_out/r06i_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06i_${tag}_${name}_${round}.json
    done
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_Q.so T=r06i STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
