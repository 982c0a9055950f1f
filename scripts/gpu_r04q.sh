# Round-4 session q: the C4 native 256^2 line (64-view set) and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04q}
B="--res 256 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_256.json 2> gpurun_out/${T}_256.log || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_256b.json 2>> gpurun_out/${T}_256.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_256 -o run --output-format csv -- python3 bench.py $B --steps 3 --warmup 1 --no-profile > gpurun_out/${T}_256p.json 2> gpurun_out/${T}_256p.log || exit 1
echo "session $T done"
