# Round-4 session m: tile sort in 3 passes of 4 bits (GSR_TILE_SORT_BITS=4: runs of ~256 keys per block and digit,
# one more pass) against 2 passes of 6 bits; bitwise tests first; runs alternated.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04m}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -k "bitwise" > gpurun_out/${T}_bitwise.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  GSR_TILE_SORT_BITS=4 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_bits4_$i.json 2> gpurun_out/${T}_bits4_$i.log || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_bits6_$i.json 2> gpurun_out/${T}_bits6_$i.log || exit 1
done
echo "session $T done"
