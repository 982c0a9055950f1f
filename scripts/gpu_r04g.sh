# Round-4 session g: blend loops with two register sets (no copies between steps), done / blend conditions as
# uniform lane masks in the forwards, the next candidate's LDS reads held ahead (GSR_FWD_PREFETCH, A/B against
# build_exp_NOPF).  Full GPU suite first.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04g}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc  # (test failures are read from the log; a crash or a time limit ends the session)
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_NOPF/libgsr_hip_exp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_nopf.json 2> gpurun_out/${T}_nopf.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.log || exit 1
# C5 backward: the two-phase quadrant walk (GSR_BWD_TW_PHASED=1) against the one-phase default
GSR_BWD_TW_PHASED=1 timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_phased.json 2> gpurun_out/${T}_c5_phased.log || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_onephase.json 2> gpurun_out/${T}_c5_onephase.log || exit 1
echo "session $T done"
