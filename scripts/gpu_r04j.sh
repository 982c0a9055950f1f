# Round-4 session j: kernel trace of the per-view drop-in path (the reference's renderer loop, one view per
# rasterizer call), 16 views per step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04j_perview -o run --output-format csv -- python3 bench.py --path per-view --views 16 --steps 2 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none --no-profile > gpurun_out/r04j_perview.json 2> gpurun_out/r04j_perview.log || exit 1
echo "session j done"
