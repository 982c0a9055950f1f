#!/bin/bash
# rocprofv3 captures for the round's profiles/ (run on the GPU box from the repo root):
#   bash profiles/run_profiles.sh <tag> [extra bench.py args, e.g. --workload sugar]
# 1) kernel trace + stats of the benchmark (bench.py's default workload unless extra args say otherwise: one
#    64-view set, 1M Gaussians, 1024^2, SH3; no secondary lines), 2) FETCH_SIZE and 3) WRITE_SIZE in separate
#    --pmc passes, 4) SQ_INSTS_VALU + SQ_WAVES (VALU roofline of the blends), each counter pass apart from
#    tracing, per the MI355X guide.  Then: python profiles/summarize.py <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04}
shift
OUT=gpurun_out/prof_${TAG}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn --extra-lines none $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT.trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/valu -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.valu.log 2>&1 || exit 1
echo "profiles $TAG done"
