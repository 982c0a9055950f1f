# Round-4 session i: what the backward's per-candidate reach-bit atomics cost (GSR_EXP_NOREACH timing library:
# wrong per-Gaussian gradients by design, render_bwd timing only), C3 and C5.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04i}
GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_NOREACH/libgsr_hip_exp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_noreach.json 2> gpurun_out/${T}_noreach.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_product.json 2> gpurun_out/${T}_product.log || exit 1
echo "session $T done"
