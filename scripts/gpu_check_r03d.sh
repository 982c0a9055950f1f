# Restored-tree check: GPU parity suite, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_gputests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || exit 1
echo done
