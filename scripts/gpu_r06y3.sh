#!/bin/bash
# Round-6 session y3: P0 (GSR_FWD_PAIR=0: HEAD's tile forward, one candidate per step, the next one's staged record
# read a step ahead) vs P2 (GSR_FWD_PAIR=2: candidates in pairs, the next pair's records read before this pair's
# arithmetic, the two power -> exp -> alpha chains issued together, then blended in list order; 94 VGPRs, 5 waves
# per SIMD), headline alternated; then the forward bitwise / parity / headline tests on P2.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2 3; do
  for spec in P0=build_ab/libgsr_hip_P0.so P2=build_ab/libgsr_hip_P2.so; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE --steps 10 --warmup 3 > gpurun_out/r06y3_v64_${name}_${round}.json \
      2> gpurun_out/r06y3_v64_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06y3_v64_${name}_${round}.json
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_P2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_configs.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06y3_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06y3_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06y3_gpu_tests.log
echo "r06y3 done"
