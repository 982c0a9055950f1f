# Round-4 session t: k_tile_ranges with the next chunk's loads in flight; tile-wave forward from 16 views.
# GPU tests, two bench runs, then the round's final counters (r04u, C3 and C5) and the default bench line
# (the driver's command) reading them.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04t}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch_renderer.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines views8"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_bench1.json 2> gpurun_out/${T}_bench.log || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_bench2.json 2>> gpurun_out/${T}_bench.log || exit 1
bash profiles/run_profiles.sh r04u || exit 1
bash profiles/run_profiles.sh r04u_sugar --workload sugar || exit 1
python profiles/summarize.py r04u > gpurun_out/r04u_summarize.log 2>&1 || exit 1
python profiles/summarize.py r04u_sugar >> gpurun_out/r04u_summarize.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --traffic profiles/r04u_traffic.json --traffic-sugar profiles/r04u_sugar_traffic.json > gpurun_out/r04u_bench_default.json 2> gpurun_out/r04u_bench_default.log || exit 1
echo "session $T done"
