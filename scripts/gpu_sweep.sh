#!/bin/bash
# GPU session: bench.py under a sweep of one environment variable.  VAR=<name> VALUES="a b c" BENCH="<args>".
mkdir -p gpurun_out
TAG=${1:-sweep}
for val in $VALUES; do
  env "$VAR=$val" timeout -k 10 200 python bench.py $BENCH > gpurun_out/${TAG}_${VAR}_${val}.json 2> gpurun_out/${TAG}_${VAR}_${val}.log || exit $?
  echo "$VAR=$val"; python scripts/bench_summary.py gpurun_out/${TAG}_${VAR}_${val}.json
done
echo done
