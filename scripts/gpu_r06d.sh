set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for spec in K=build_ab/libgsr_hip_K.so L=build_ab/libgsr_hip_L.so; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/r06d_sugar_${name}_${round}.json 2> gpurun_out/r06d_sugar_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06d_sugar_${name}_${round}.json
  done
done
T=r06d STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
