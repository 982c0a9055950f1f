# Round-4 session k: the lockstep backward's cull from the tile-wave forward's masks; full GPU suite, bench A/B
# (GSR_FWD_KERNEL=quadrant takes the forward without masks at C3: an upper bound on what the masks save).
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04k}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.log || exit 1
echo "session $T done"
