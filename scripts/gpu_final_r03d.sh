# Round-3 final GPU session (session d): parity suite, smoke, bench lines, kernel traces (default C3 line and C5).
set -o pipefail
mkdir -p gpurun_out
T=r03d
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_final_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_final_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_final_bench.json 2> gpurun_out/${T}_final_bench.log || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/${T}_final_sugar.json 2> gpurun_out/${T}_final_sugar.log || exit 1
timeout -k 10 300 python -u bench.py --epilogue shading --no-cpu-baseline --no-knn > gpurun_out/${T}_final_shading.json 2> gpurun_out/${T}_final_shading.log || exit 1
timeout -k 10 300 python -u bench.py --res 256 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_final_256.json 2> gpurun_out/${T}_final_256.log || exit 1
timeout -k 10 300 python -u bench.py --views 8 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_final_v8.json 2> gpurun_out/${T}_final_v8.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${T}_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_sugar/trace -o run --output-format csv -- python3 bench.py $ARGS --workload sugar > gpurun_out/${T}_trace_sugar.log 2>&1 || exit 1
echo done
