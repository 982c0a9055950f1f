# Round-4 session b: the two-colour tile-wave backward vs the lockstep one (diagnostic), the parity suite
# (failures recorded, not fatal), smoke, the default bench and its A/B variants, the --gpus 2 launcher rehearsal
# on one GPU, counters of the C3 and C5 blends.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04b}
timeout -k 10 200 python -u scripts/diag_bwd_tw.py two > gpurun_out/${T}_diag_tw.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/diag_bwd_tw.py one >> gpurun_out/${T}_diag_tw.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_FWD_KERNEL=quadrant GSR_BWD_KERNEL=quadrant timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_bench_quadrant.json 2> gpurun_out/${T}_bench_quadrant.log || exit 1
GSR_BWD_KERNEL=quadrant timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_bench_bwdquad.json 2> gpurun_out/${T}_bench_bwdquad.log || exit 1
GSR_BENCH_SHARE_GPU=1 GSR_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-knn > gpurun_out/${T}_gpus2.json 2> gpurun_out/${T}_gpus2.log || exit 1
bash profiles/run_profiles.sh ${T} || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
