#!/bin/bash
# Round-6 session x2: B0 (HEAD) vs PK (the tile-wave forward forms (B dy, C dy) as one packed product and (dx, dy)
# as one packed difference, as the quadrant-wave forward does: 2 fewer VALU instructions per (candidate, quadrant)
# step, the same IEEE operations; the epilogue re-derives its pixel row so nothing spills), headline and 256^2 alternated; then the forward bitwise / parity tests on PK.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2 3; do
  for spec in B0=build_ab/libgsr_hip_B0.so PK=build_ab/libgsr_hip_PK2.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "r256:--res 256 --steps 10 --warmup 3"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06x2_${tag}_${name}_${round}.json \
        2> gpurun_out/r06x2_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06x2_${tag}_${name}_${round}.json
    done
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_PK2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_configs.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06x2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06x2_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06x2_gpu_tests.log
echo "r06x2 done"
