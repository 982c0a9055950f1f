# Round-4 session r: kernel trace of the 8-view set (the N = 8 per-rank share) for its fixed costs.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--views 8 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_v8 -o run --output-format csv -- python3 bench.py $B --steps 8 --warmup 2 --no-profile > gpurun_out/${T}_v8p.json 2> gpurun_out/${T}_v8p.log || exit 1
echo "session $T done"
