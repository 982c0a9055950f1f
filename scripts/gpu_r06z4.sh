#!/bin/bash
# Round-6 session z4: other build-time tunables re-swept on the final kernels against HEAD (CH8 = the in-tree
# configuration): EG1 / EG4 = GSR_EMIT_GROUPS 1 / 4 (64-Gaussian emission groups per wave, HEAD 2), OV2 = GSR_BWD_OVERLAP 2
# (HEAD 1; spills 4 VGPRs), VI8 = GSR_VG_ITEMS 8 (HEAD 16); headline alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for name in CH8 EG1 EG4 OV2 VI8; do
    GSR_HIP_LIB=$PWD/build_ab/libgsr_hip_$name.so timeout -k 10 300 python -u bench.py $BASE --steps 10 --warmup 3 \
      > gpurun_out/r06z4_v64_${name}_${round}.json 2> gpurun_out/r06z4_v64_${name}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06z4_v64_${name}_${round}.json
  done
done
echo "r06z4 done"
