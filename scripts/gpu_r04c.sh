# Round-4 session c: the one-wave-per-tile backward kernels (hit lists for C5, matrix cores for C3) vs the lockstep
# workgroup: bitwise diagnostics, the parity suite, smoke, bench A/B, counters of the new default kernels.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04c}
timeout -k 10 200 python -u scripts/diag_bwd_tw.py two > gpurun_out/${T}_diag_tw.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/diag_bwd_tw.py one >> gpurun_out/${T}_diag_tw.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/diag_bwd_tw.py one hits >> gpurun_out/${T}_diag_tw.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_BWD_KERNEL=quadrant timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench_bwdquad.json 2> gpurun_out/${T}_bench_bwdquad.log || exit 1
GSR_FWD_KERNEL=tq timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench_tq.json 2> gpurun_out/${T}_bench_tq.log || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
bash profiles/run_profiles.sh ${T} || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
