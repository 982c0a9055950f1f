#!/bin/bash
# Round-6 session g: N (in-tree) vs O (two-colour tile-wave backward with one wait point per batch) on the C5 SuGaR
# set, then O's two-colour parity tests and the whole gpu suite on O.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in N=build_ab/libgsr_hip_N.so O=build_ab/libgsr_hip_O.so; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE --workload sugar --steps 5 --warmup 2 \
      > gpurun_out/r06g_c5_${name}_${round}.json 2> gpurun_out/r06g_c5_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06g_c5_${name}_${round}.json
  done
done
GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_O.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r06g_tests_O.log 2>&1 || { tail -30 gpurun_out/r06g_tests_O.log; exit 1; }
tail -3 gpurun_out/r06g_tests_O.log
echo "r06g done"
