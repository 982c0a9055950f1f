#!/bin/bash
# GPU session: split backward on / off (GSR_BWD_SPLIT=0) alternated on the per-view path (one-view launches).
mkdir -p gpurun_out
TAG=${1:-split_ab}
B="--no-cpu-baseline --no-knn --per-view-views 0 --path per-view --views 16 --steps 4 --warmup 1"
for rep in 1 2; do
  for mode in on off; do
    if [ $mode = off ]; then export GSR_BWD_SPLIT=0; else unset GSR_BWD_SPLIT; fi
    timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_pv_${mode}_${rep}.json 2>> gpurun_out/${TAG}.log || exit $?
    echo "rep $rep $mode done"
  done
done
for f in gpurun_out/${TAG}_*.json; do python scripts/bench_summary.py $f; done
