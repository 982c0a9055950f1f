set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch_renderer.py -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r02_sugar_tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/r02_sugar_tests.log
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/r02_bench_sugar.json 2> gpurun_out/r02_bench_sugar.log || exit 1
GSR_BENCH_SUGAR_SEPARATE=1 timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/r02_bench_sugar_sep.json 2> gpurun_out/r02_bench_sugar_sep.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/r02_bench_check.json 2> gpurun_out/r02_bench_check.log
