#!/bin/bash
# Round-6 final build 6ef9dfa6a022 (per-launch dispatch-order chunks), part 1: the driver's default bench line, the
# C5 line, 64 views at 256^2 (the gpu suite ran on this build in session r06z6).
set -o pipefail
mkdir -p gpurun_out
T=r06g STEPS="bench sugar" bash scripts/gpu_session.sh || exit 1
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 python -u bench.py $BASE --res 256 --steps 10 --warmup 3 > gpurun_out/r06g_256.json 2> gpurun_out/r06g_256.log || exit 1
python scripts/bench_summary.py gpurun_out/r06g_256.json
echo "r06g1 done"
