# Round-4 session v: per-tile list bounds by search (k_tile_bounds) instead of a scan of every sorted key.
# Bitwise switch tests + parity; C3 / 8-view A/B (runs alternated); kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5,views8"
for r in 1 2; do
  GSR_TILE_RANGES=scan timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_scan$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_search$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn --extra-lines none --no-profile > gpurun_out/${T}_trace.log 2>&1 || exit 1
echo "session $T done"
