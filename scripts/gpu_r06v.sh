#!/bin/bash
# Round-6 final build c1fce774b792 (the committed sources of 285f60d; the library profiled in session r06z,
# 31ab57896994, had been built from an uncommitted state of the tree): the whole -m gpu suite, the driver's default
# bench line, C5, 64 views at 256^2, then the kernel trace + FETCH / WRITE / VALU passes of C3 and C5,
# device-counted pairs (diagnostic build of the same sources) and the SQ counters of the C3 blends.
set -o pipefail
mkdir -p gpurun_out
T=r06v STEPS="tests bench sugar" bash scripts/gpu_session.sh || exit 1
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 python -u bench.py $BASE --res 256 --steps 10 --warmup 3 > gpurun_out/r06v_256.json 2> gpurun_out/r06v_256.log || exit 1
python scripts/bench_summary.py gpurun_out/r06v_256.json
T=r06v STEPS="prof profsugar pairs sq" bash scripts/gpu_session.sh || exit 1
echo "r06v done"
