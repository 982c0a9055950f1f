#!/bin/bash
# Round-6 session n: C5 with the tile-wave forward forced (GSR_FWD_KERNEL=tile) against the default quadrant-wave
# forward, alternated; then where the secondary lines stand: 64 views at 256^2 and the per-view path.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for k in default tile; do
    if [ $k = tile ]; then export GSR_FWD_KERNEL=tile; else unset GSR_FWD_KERNEL; fi
    timeout -k 10 300 python -u bench.py $BASE --workload sugar --steps 5 --warmup 2 > gpurun_out/r06n_c5_${k}_${round}.json \
      2> gpurun_out/r06n_c5_${k}_${round}.log || exit 1
    python scripts/bench_summary.py gpurun_out/r06n_c5_${k}_${round}.json
  done
done
unset GSR_FWD_KERNEL
timeout -k 10 300 python -u bench.py $BASE --res 256 --steps 10 --warmup 3 > gpurun_out/r06n_256.json 2> gpurun_out/r06n_256.log || exit 1
python scripts/bench_summary.py gpurun_out/r06n_256.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --extra-lines none --path per-view --views 16 --steps 3 --warmup 1 \
  > gpurun_out/r06n_pv.json 2> gpurun_out/r06n_pv.log || exit 1
python scripts/bench_summary.py gpurun_out/r06n_pv.json
echo "r06n done"
