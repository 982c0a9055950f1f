# Round-4 session zz: the final tree's N = 2 path (two ranks sharing the box's GPU over gloo: the launcher, view
# sharding and the gathered / reduced step), the 256^2 line, and 64 views per preprocess block
# (build_ab/libgsr_hip_pre64.so, -DGSR_PRE_VIEWS=64) against 32 (runs alternated; parity tests on the variant).
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zz}
GSR_BENCH_SHARE_GPU=1 GSR_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-knn > gpurun_out/${T}_gpus2.json 2> gpurun_out/${T}_gpus2.log || exit 1
timeout -k 10 300 python -u bench.py --res 256 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/${T}_256.json 2> gpurun_out/${T}_256.log || exit 1
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_pre64.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pre64_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_pre32_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
  GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_pre64.so timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_pre64_$r.json 2>> gpurun_out/${T}_bench.log || exit 1
done
echo "session $T done"
