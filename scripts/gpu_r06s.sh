#!/bin/bash
# Round-6 session s: the per-view drop-in path (bench.py --path per-view: one GaussianRasterizer call per view,
# 64 views per step) with NP1 (the working tree built with GSR_EXP_NOPRE1: one-view sets take the 64-view-block
# preprocess, half its waves idle) vs P1 (one-view sets: a thread per Gaussian, SH read from HBM), alternated;
# then the parity tests on P1.
set -o pipefail
mkdir -p gpurun_out
BASE="--path per-view --steps 5 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2 3; do
  for spec in NP1=build_ab/libgsr_hip_NP1.so P1=build_ab/libgsr_hip_P1.so; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE > gpurun_out/r06s_pv_${name}_${round}.json \
      2> gpurun_out/r06s_pv_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06s_pv_${name}_${round}.json
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_P1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06s_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06s_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06s_gpu_tests.log
echo "r06s done"
