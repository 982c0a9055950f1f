#!/bin/bash
# GPU session: rocprofv3 kernel trace + stats of one bench.py configuration: ARGS="<bench args>".
mkdir -p gpurun_out
TAG=${1:-trace}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o run --output-format csv -- python3 bench.py $ARGS --no-profile > gpurun_out/${TAG}.log 2>&1 || exit $?
echo done
