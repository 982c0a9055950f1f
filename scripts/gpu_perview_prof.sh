# Kernel trace of the drop-in per-view path (one GaussianRasterizer call per view), timing only.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_prof -o pv --output-format csv -- python3 bench.py --path per-view --views 16 --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/pv_bench.json 2> gpurun_out/pv_bench.log || exit 1
find gpurun_out/pv_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/pv_kernel_stats.csv \;
