# Round-4 session c5f: kernel trace of the C5 line (SuGaR normal renderer) on the final tree.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04c5f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --workload sugar --steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn --extra-lines none --no-profile > gpurun_out/${T}_trace.log 2>&1 || exit 1
echo "session $T done"
