#!/bin/bash
# Round-6 final build 347b41455d76, part 3: the whole -m gpu suite, then the driver's default bench line with the
# build's own counters (profiles/r06h_*) attached.
set -o pipefail
mkdir -p gpurun_out
T=r06h3 STEPS="tests bench" bash scripts/gpu_session.sh || exit 1
echo "r06h3 done"
