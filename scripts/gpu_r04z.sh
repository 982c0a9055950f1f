# Round-4 session z: occupancy of two binning kernels — k_emit<false> without the mask-only LDS arrays (4.6 KB:
# 8 instead of 7 single-wave workgroups per SIMD) and the keys-only sort scatter at 6 waves per SIMD (80 VGPRs) —
# = the default library, vs the tree before them (build_ab/libgsr_hip_base.so); runs alternated.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04z}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines views8"
for r in 1 2 3; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_base.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_base_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_new_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
echo "session $T done"
