# Round-4 session f: SQ counters (wave cycles / waits / issue, LDS, VALU) of the three blend kernels that bound
# the step: C3 forward (k_render_fwd_tile<false>) and backward (k_render_bwd<false, false>) over a 64-view set,
# C5 backward (k_render_bwd_tw<true, 1>) over a 16-view set.  profiles/run_sq.sh runs one --pmc pass per group.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/r04f_c5.json 2> gpurun_out/r04f_c5.log || exit 1
SQ_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-knn --per-view-views 0 --extra-lines none" bash profiles/run_sq.sh r04c3 || exit 1
python profiles/sq_summary.py r04c3 "k_render_fwd_tile<false>" > gpurun_out/sq_r04c3_fwd.txt || exit 1
python profiles/sq_summary.py r04c3 "k_render_bwd<false, false>" > gpurun_out/sq_r04c3_bwd.txt || exit 1
SQ_ARGS="--workload sugar --views 16 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-knn --per-view-views 0 --extra-lines none" bash profiles/run_sq.sh r04c5 || exit 1
python profiles/sq_summary.py r04c5 "k_render_bwd_tw<true, 1>" > gpurun_out/sq_r04c5_bwd.txt || exit 1
python profiles/sq_summary.py r04c5 "k_render_fwd<true, false>" > gpurun_out/sq_r04c5_fwd.txt || exit 1
echo "session f done"
