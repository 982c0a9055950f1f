#!/bin/bash
# GPU session: parity tests; then (only if pytest ended normally) optional extra steps.
mkdir -p gpurun_out
TAG=${1:-r03_gpu}
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -s ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 240 python bench.py $BENCH > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
fi
echo done
