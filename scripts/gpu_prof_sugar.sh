# rocprofv3 captures of the C5 line (bench.py --workload sugar): kernel trace, FETCH_SIZE, WRITE_SIZE and
# SQ_INSTS_VALU / SQ_WAVES in separate passes -> gpurun_out/prof_r03d_sugar (profiles/summarize.py r03d_sugar).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/prof_r03d_sugar
ARGS="--workload sugar --steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT.trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $OUT/valu -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT.valu.log 2>&1 || exit 1
echo done
