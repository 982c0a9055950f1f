#!/bin/bash
# GPU session: the drop-in per-view path (one GaussianRasterizer call per view): bench line with host trace,
# then a kernel trace of the same command.
mkdir -p gpurun_out
TAG=${1:-perview}
ARGS="--path per-view --views 16 --steps 4 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0"
GSR_HOST_TRACE=1 timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.log || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- python3 bench.py $ARGS --no-profile > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
python scripts/bench_summary.py gpurun_out/${TAG}.json
echo done
