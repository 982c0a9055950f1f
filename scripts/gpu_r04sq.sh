# Round-4 session sq: SQ counters of the final tree's C3 blends (one --pmc pass per group) for DESIGN §8's table.
set -o pipefail
mkdir -p gpurun_out
SQ_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-knn --per-view-views 0 --extra-lines none" bash profiles/run_sq.sh r04fin || exit 1
python profiles/sq_summary.py r04fin "k_render_fwd_tile<false>" > gpurun_out/sq_r04fin_fwd.txt || exit 1
python profiles/sq_summary.py r04fin "k_render_bwd<false, false>" > gpurun_out/sq_r04fin_bwd.txt || exit 1
echo "session sq done"
