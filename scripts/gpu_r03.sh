#!/bin/bash
# GPU session: parity tests; then (only if pytest ended normally: passed or assertion failures) the optional
# steps named by the environment: BENCH="<bench.py args>" (one bench run), MICRO=1 (MFMA rate microbenchmark).
mkdir -p gpurun_out
TAG=${1:-r03_gpu}
if [ -z "$NOTEST" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -s ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}.log 2>&1
  rc=$?
  echo "pytest rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$MICRO" ]; then
  timeout -k 10 60 ./profiles/microbench/mfma_rates > gpurun_out/${TAG}_mfma.txt 2>&1 || exit $?
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py $BENCH > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
fi
echo done
