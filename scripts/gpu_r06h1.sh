#!/bin/bash
# Round-6 final build (per-launch dispatch-order chunks, small chunks only for sets of >= 32 views of >= 512
# super-tiles), part 1: the oracle / bitwise / headline / config tests, the driver's default bench line, the C5
# line, 64 views at 256^2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r06h_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06h_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06h_gpu_tests.log
T=r06h STEPS="bench sugar" bash scripts/gpu_session.sh || exit 1
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 python -u bench.py $BASE --res 256 --steps 10 --warmup 3 > gpurun_out/r06h_256.json 2> gpurun_out/r06h_256.log || exit 1
python scripts/bench_summary.py gpurun_out/r06h_256.json
echo "r06h1 done"
