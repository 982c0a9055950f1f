#!/bin/bash
# Round-6 final build, part 2: rocprofv3 kernel trace + FETCH / WRITE / VALU passes of the C3 and C5
# workloads, device-counted pairs (diagnostic build of the same sources), SQ counters of the C3 blends.
set -o pipefail
mkdir -p gpurun_out
T=r06h STEPS="prof profsugar pairs sq" bash scripts/gpu_session.sh
