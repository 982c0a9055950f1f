# Round-4 session n: packed fp32 pairs in the forward blends. Bitwise / forward tests, then bench (C3, C5, views8).
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.log || exit 1
echo "session $T done"
