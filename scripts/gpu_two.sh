# Two-colour backward (one pass for both SuGaR calls): parity tests, then the C5 bench fused vs separate.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch_renderer.py -m gpu -v -s -rf --timeout 600 --timeout-method thread -k "second_colors or c5 or sugar" > gpurun_out/two_tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/two_tests.log
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/two_bench_sugar.json 2> gpurun_out/two_bench_sugar.log || exit 1
GSR_TWO_COLOR_BWD=separate timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/two_bench_sugar_sep.json 2> gpurun_out/two_bench_sugar_sep.log
