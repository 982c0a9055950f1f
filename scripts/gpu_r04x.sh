# Round-4 session x (and the round's last, T=r04final): the final tree — full GPU suite, smoke, the default bench
# line (the driver's command) and a kernel trace of the benchmark.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04x}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn --extra-lines none --no-profile > gpurun_out/${T}_trace.log 2>&1 || exit 1
echo "session $T done"
