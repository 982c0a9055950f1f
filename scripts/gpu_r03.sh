#!/bin/bash
# Round-3 GPU session: parity tests, then (only if pytest ended normally: all passed or assertion failures)
# the pair counters and one bench run.  Any other exit (fault, abort, timeout) ends the session.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s > gpurun_out/r03_gpu1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python profiles/diag_pairs.py r03 > gpurun_out/r03_pairs.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > gpurun_out/r03_bench1.json 2> gpurun_out/r03_bench1.log || exit $?
echo done
