# Round-4 session y: k_gauss_accum at 3 waves per SIMD (SH row read from LDS where used, two record buffers; 7
# VGPRs spilled outside the view loop) = the default library, vs the product build before it
# (build_ab/libgsr_hip_v0.so) and vs the same plus k_view_grad<false> at 5 waves per SIMD
# (build_ab/libgsr_hip_v3.so; 3 VGPRs spilled, one reload per item); runs alternated.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04y}
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_batch_renderer.py tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines views8"
for r in 1 2; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_v0.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_v0_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_v2_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_v3.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_v3_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
echo "session $T done"
