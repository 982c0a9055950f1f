#!/bin/bash
# Round-6 final session, part 1 (the final build): the whole -m gpu suite, the driver's default bench line, the C5
# line, 64 views at 256^2 and the per-view path.
set -o pipefail
mkdir -p gpurun_out
T=r06x STEPS="tests bench sugar" TEST_TIMEOUT=300 bash scripts/gpu_session.sh || exit 1
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 python -u bench.py $BASE --res 256 --steps 10 --warmup 3 > gpurun_out/r06x_256.json 2> gpurun_out/r06x_256.log || exit 1
python scripts/bench_summary.py gpurun_out/r06x_256.json
echo "r06x1 done"
