#!/bin/bash
# Round-6 session w: NX4 (the working tree built with GSR_EXP_NOX4: the sort's count kernel loads its 16 keys per
# lane as 16 dword loads, as HEAD) vs X4 (16-byte loads, 1 KB per wave instruction, for 16-B aligned segments),
# headline and C5 alternated; then the sort and parity tests on X4.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in NX4=build_ab/libgsr_hip_NX4.so X4=build_ab/libgsr_hip_X4.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "c5:--workload sugar --steps 10 --warmup 3"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06w_${tag}_${name}_${round}.json \
        2> gpurun_out/r06w_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06w_${tag}_${name}_${round}.json
    done
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_X4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_parity.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06w_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06w_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06w_gpu_tests.log
echo "r06w done"
