# Round-3 (session d) check: GPU parity suite, smoke, the default bench line and the C5 / shading lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_gputests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/r03d_bench_sugar.json 2> gpurun_out/r03d_bench_sugar.err || exit 1
echo done
