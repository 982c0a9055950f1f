# Round-4 session p: 1024-pair sort blocks for small sets (one view's depth sort, the 3-NN sort), LDS-staged
# kept-count scan.  Bitwise switch tests + KNN + parity; per-view A/B (runs alternated); per-view kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_knn.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
PV="--path per-view --views 16 --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for r in 1 2; do
  GSR_SORT_SMALL_PAIRS=0 timeout -k 10 300 python -u bench.py $PV > gpurun_out/${T}_pv_big$r.json 2>> gpurun_out/${T}_pv.log || exit 1
  timeout -k 10 300 python -u bench.py $PV > gpurun_out/${T}_pv_small$r.json 2>> gpurun_out/${T}_pv.log || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_perview -o run --output-format csv -- python3 bench.py --path per-view --views 16 --steps 2 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none --no-profile > gpurun_out/${T}_perview.json 2> gpurun_out/${T}_perview.log || exit 1
echo "session $T done"
