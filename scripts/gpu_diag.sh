set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/diag_tile.py > gpurun_out/r02_diag_tile.log 2>&1
