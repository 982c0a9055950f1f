#!/bin/bash
# Round-6 session o: NE (the working tree built with GSR_EXP_NOEMBED: the two-colour blends gather colors2 apart, as
# HEAD does) vs E (the second colours embedded in the records by the preprocess, gsr_set_preprocess_ex, read from
# the record line), C5 alternated; then the whole gpu suite on the in-tree library (= E).
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in NE=build_ab/libgsr_hip_NE.so E=build_ab/libgsr_hip_E.so; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE --workload sugar --steps 5 --warmup 2 \
      > gpurun_out/r06o_c5_${name}_${round}.json 2> gpurun_out/r06o_c5_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06o_c5_${name}_${round}.json
  done
done
T=r06o STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
