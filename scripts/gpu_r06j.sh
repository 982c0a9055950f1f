#!/bin/bash
# Round-6 session j: the sort scatter's in-wave ranking per pass — P (HEAD: ballot matching everywhere) vs U (ballot,
# per-wave digit starts folded: one LDS read per item per phase) vs S (U + LDS-atomic ranks in the tile sort's first
# pass) vs T (U + LDS-atomic ranks in both tile-sort passes), on the headline, the 8-view set and C5; then the GPU
# sort tests on S and T.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in P=build_ab/libgsr_hip_P.so U=build_ab/libgsr_hip_U.so S=build_ab/libgsr_hip_S.so T=build_ab/libgsr_hip_T.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06j_${tag}_${name}_${round}.json \
        2> gpurun_out/r06j_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06j_${tag}_${name}_${round}.json
    done
  done
done
for name in S T U; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r06j_sort_$name.log 2>&1 || { tail -30 gpurun_out/r06j_sort_$name.log; exit 1; }
  tail -1 gpurun_out/r06j_sort_$name.log
done
echo "r06j done"
