# SQ counters of the C5 two-colour hit-list backward blend (16-view set, 4 --pmc passes) and, for comparison,
# the matrix-core variant (GSR_BWD_SUMS=mfma).
set -o pipefail
mkdir -p gpurun_out
SQ_ARGS="--workload sugar --steps 1 --warmup 1 --views 16 --no-cpu-baseline --no-profile --no-knn --per-view-views 0" bash profiles/run_sq.sh c5hits || exit 1
python profiles/sq_summary.py c5hits "k_render_bwd<true, true>" > gpurun_out/sq_c5hits.txt || exit 1
GSR_BWD_SUMS=mfma SQ_ARGS="--workload sugar --steps 1 --warmup 1 --views 16 --no-cpu-baseline --no-profile --no-knn --per-view-views 0" bash profiles/run_sq.sh c5mfma || exit 1
python profiles/sq_summary.py c5mfma "k_render_bwd<true, false>" > gpurun_out/sq_c5mfma.txt || exit 1
echo done
