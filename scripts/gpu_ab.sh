#!/bin/bash
# GPU session: A/B of library builds in one session, alternated: LIBS="name=path ..." BENCH="<bench args>".
mkdir -p gpurun_out
TAG=${1:-ab}
for round in 1 2; do
  for spec in $LIBS; do
    name=${spec%%=*}; lib=${spec#*=}
    GSR_HIP_LIB=$lib timeout -k 10 200 python bench.py $BENCH > gpurun_out/${TAG}_${name}_${round}.json 2> gpurun_out/${TAG}_${name}_${round}.log || exit $?
    python scripts/bench_summary.py gpurun_out/${TAG}_${name}_${round}.json
  done
done
echo done
