# Round-4 session l: one-view preprocess and range-block changes; full GPU suite; the default bench line exactly
# as the driver runs it (no flags); per-view path kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04l}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_perview -o run --output-format csv -- python3 bench.py --path per-view --views 16 --steps 2 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none --no-profile > gpurun_out/${T}_perview.json 2> gpurun_out/${T}_perview.log || exit 1
echo "session $T done"
