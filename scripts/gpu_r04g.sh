# Round-4 session g: tile-wave backward replay unrolled by two (no register copies between steps); forward
# blends with the next candidate's LDS reads held ahead (GSR_FWD_PREFETCH, A/B against build_exp_NOPF).
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -k "bitwise" > gpurun_out/${T}_bitwise.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_NOPF/libgsr_hip_exp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_nopf.json 2> gpurun_out/${T}_nopf.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 8 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.log || exit 1
echo "session $T done"
