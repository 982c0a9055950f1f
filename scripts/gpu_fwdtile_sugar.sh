# C5 forward: tile-wave kernel (one gather per candidate per tile; GSR_FWD_KERNEL=tile) vs the quadrant-wave
# product, one session alternated.
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/fwdtile_sugar.txt
: > $OUTF
for round in 1 2; do
for K in quadrant tile; do
  GSR_FWD_KERNEL=$K timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/ft_$K.json 2> gpurun_out/ft_$K.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ft_$K.json')); print('sugar', '$K', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
