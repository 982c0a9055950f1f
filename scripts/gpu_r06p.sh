#!/bin/bash
# Round-6 session p: the count kernel's histogram spread over padded copies (lane mod N): C1 = HEAD (one histogram),
# C8 = 8 copies, C4 = 4 copies; the headline and C5 (whose second tile-sort count pass ran 4x its first: runs of
# equal digits), alternated; then the GPU sort tests on C8 and C4.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in C1=build_ab/libgsr_hip_C1.so C8=build_ab/libgsr_hip_C8.so C4=build_ab/libgsr_hip_C4.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06p_${tag}_${name}_${round}.json \
        2> gpurun_out/r06p_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06p_${tag}_${name}_${round}.json
    done
  done
done
for name in C8 C4; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r06p_sort_$name.log 2>&1 || { tail -30 gpurun_out/r06p_sort_$name.log; exit 1; }
  tail -1 gpurun_out/r06p_sort_$name.log
done
echo "r06p done"
