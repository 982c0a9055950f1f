#!/bin/bash
# Round-6 final build 285f60d: bench lines (part 1) then the profiles (part 2) in one call.
set -o pipefail
bash scripts/gpu_r06z1.sh && bash scripts/gpu_r06z2.sh
