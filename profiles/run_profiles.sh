#!/bin/bash
# rocprofv3 captures for the round's profiles/ (run on the GPU box from the repo root):
#   bash profiles/run_profiles.sh <tag>
# 1) kernel trace + stats of the benchmark (same workload as bench.py's defaults: 64-view set,
#    1M Gaussians, 1024^2, SH3), 2) FETCH_SIZE and 3) WRITE_SIZE in separate --pmc passes
# 4) SQ_INSTS_VALU + SQ_WAVES (VALU roofline of the blends), each counter pass apart from tracing, per the
# MI355X guide.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${1:-r01}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT.trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/valu -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.valu.log 2>&1
echo done
