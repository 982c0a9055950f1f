# Round-4 session s: forward kernel choice for small sets (8 / 16 / 32 views): tile-wave vs quadrant-wave, runs
# alternated.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04s}
for V in 8 16 32; do
  B="--views $V --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none --steps 8 --warmup 2"
  for r in 1 2; do
    GSR_FWD_KERNEL=quadrant timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_v${V}_quad$r.json 2>> gpurun_out/${T}.log || exit 1
    GSR_FWD_KERNEL=tile timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_v${V}_tile$r.json 2>> gpurun_out/${T}.log || exit 1
  done
done
echo "session $T done"
