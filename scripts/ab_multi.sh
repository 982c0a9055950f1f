#!/bin/bash
# A/B of library builds over several bench.py workloads (run on the GPU box from the repo root):
#   T=<tag> LIBS="name=path ..." ROUNDS=2 bash scripts/ab_multi.sh
# Workloads: the default 64-view line, 8-view sets, the per-view drop-in path (16 views).  Each run under its own
# time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in $(seq 1 ${ROUNDS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5" "pv:--path per-view --views 16 --steps 3 --warmup 1"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/${T}_${tag}_${name}_${round}.json \
        2> gpurun_out/${T}_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/${T}_${tag}_${name}_${round}.json
    done
  done
done
echo "ab_multi $T done"
