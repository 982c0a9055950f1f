# Round-4 session e: quadrant masks in the unpacked keys (span_quads per row in k_emit), one-wave tile backward by
# default, fused per-Gaussian backward without SH only.  Full GPU suite, bench, masks A/B, C5 counters.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_TILE_KEYS=plain timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_plain.json 2> gpurun_out/${T}_c5_plain.log || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_masks.json 2> gpurun_out/${T}_c5_masks.log || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
