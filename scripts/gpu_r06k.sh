#!/bin/bash
# Round-6 session k: the in-tree library with LDS-atomic ranks in both tile-sort passes (T) behind the lane-order
# probe: the whole gpu suite (incl. the probe and ballot-fallback tests), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
T=r06k STEPS="tests bench" TEST_TIMEOUT=300 bash scripts/gpu_session.sh
