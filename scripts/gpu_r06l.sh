#!/bin/bash
# Round-6 session l: H16 (HEAD 16244e7) vs X (count kernel over 4 blocks per workgroup, the next block's keys loaded
# while the current one is counted) vs Y (X + LDS-atomic ranks in the depth sort's first key/value pass), on the
# headline, the 8-view set and C5; then the GPU sort tests on X and Y.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in H16=build_ab/libgsr_hip_H16.so X=build_ab/libgsr_hip_X.so Y=build_ab/libgsr_hip_Y.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5" "c5:--workload sugar --steps 5 --warmup 2"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06l_${tag}_${name}_${round}.json \
        2> gpurun_out/r06l_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06l_${tag}_${name}_${round}.json
    done
  done
done
for name in X Y; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r06l_sort_$name.log 2>&1 || { tail -30 gpurun_out/r06l_sort_$name.log; exit 1; }
  tail -1 gpurun_out/r06l_sort_$name.log
done
echo "r06l done"
