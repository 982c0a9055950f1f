#!/bin/bash
# GPU session: the default bench line (the driver's command) and the side lines DESIGN.md quotes.
mkdir -p gpurun_out
TAG=${1:-lines}
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.log || exit $?
timeout -k 10 200 python bench.py --res 256 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${TAG}_256.json 2> gpurun_out/${TAG}_256.log || exit $?
timeout -k 10 200 python bench.py --views 8 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${TAG}_v8.json 2> gpurun_out/${TAG}_v8.log || exit $?
timeout -k 10 200 python bench.py --epilogue shading --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${TAG}_shading.json 2> gpurun_out/${TAG}_shading.log || exit $?
python scripts/bench_summary.py gpurun_out/${TAG}_*.json
echo done
