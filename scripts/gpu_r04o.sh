# Round-4 session o: means2D gradient in an explicit operation order (tile-wave packed replay bitwise again).
# Full GPU suite, then the default bench.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04o}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
echo "session $T done"
