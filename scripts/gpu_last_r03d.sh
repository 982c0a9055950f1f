# Last check of the round's tree: full GPU suite, smoke, default and C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/r03d_last_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_last_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03d_last_bench.json 2> gpurun_out/r03d_last_bench.log || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/r03d_last_sugar.json 2> gpurun_out/r03d_last_sugar.log || exit 1
echo done
