# Round-4 session w: wave-cooperative kept-tile rows in the preprocess (GSR_PRE_ROWS=wave|lane).
# Parity / config tests; A/B at C3, 256^2 and the 8-view set (runs alternated).
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04w}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines views8"
B2="--res 256 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for r in 1 2; do
  GSR_PRE_ROWS=lane timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_lane$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_wave$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  GSR_PRE_ROWS=lane timeout -k 10 300 python -u bench.py $B2 > gpurun_out/${T}_lane256_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  timeout -k 10 300 python -u bench.py $B2 > gpurun_out/${T}_wave256_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
echo "session $T done"
