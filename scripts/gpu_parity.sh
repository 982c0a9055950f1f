# GPU parity run: all -m gpu tests with the adjudication report (-s), one process.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rf --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/r02_parity.log 2>&1
echo "pytest exit $?" >> gpurun_out/r02_parity.log
