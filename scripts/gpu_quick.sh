# Parity suite + C3 / C5 bench lines after a kernel change.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1
echo "pytest exit $?" >> gpurun_out/${TAG}_parity.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_bench$i.log || exit 1
done
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/${TAG}_bench_sugar.json 2> gpurun_out/${TAG}_bench_sugar.log
