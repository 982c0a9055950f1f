#!/bin/bash
# Round-6 session q: the renderers' clamp(0, 1) formed in the blends (rasterize_views clamp=True; gsr_set_render_*
# with out_render but no bg_images): C5 with --fused-clamp off (torch clamp on the colour output) vs on, on the
# working tree's library (in-tree), alternated; the headline once; then the whole gpu suite.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for fc in off on; do
    timeout -k 10 300 python -u bench.py $BASE --workload sugar --steps 5 --warmup 2 --fused-clamp $fc \
      > gpurun_out/r06q_c5_${fc}_${round}.json 2> gpurun_out/r06q_c5_${fc}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06q_c5_${fc}_${round}.json
  done
done
timeout -k 10 300 python -u bench.py $BASE --steps 10 --warmup 3 > gpurun_out/r06q_v64.json 2> gpurun_out/r06q_v64.log || exit 1
python scripts/bench_summary.py gpurun_out/r06q_v64.json
T=r06q STEPS="tests" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
