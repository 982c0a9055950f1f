# Bench lines of the round (default = the metric's line), plus the C5 / shading workloads and C5 pair counts.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit 1
timeout -k 10 400 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/${TAG}_bench_sugar.json 2> gpurun_out/${TAG}_bench_sugar.log || exit 1
timeout -k 10 400 python -u bench.py --epilogue shading --no-cpu-baseline --no-knn > gpurun_out/${TAG}_bench_shading.json 2> gpurun_out/${TAG}_bench_shading.log || exit 1
timeout -k 10 300 python -u profiles/diag_pairs.py $TAG sugar > gpurun_out/${TAG}_pairs_sugar.log 2>&1
