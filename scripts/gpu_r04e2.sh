# Round-4 session e2: 64-Gaussian groups per k_emit wave — 2 (default) vs 4 and 1 (build_ab/libgsr_hip_eg{4,1}.so,
# -DGSR_EMIT_GROUPS); parity tests on each variant, then runs alternated.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04e2}
for v in eg4 eg1; do
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_${v}_tests.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
done
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines views8"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_eg2_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_eg4.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_eg4_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_eg1.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_eg1_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
echo "session $T done"
