# Hit-list sums in the backward blend: parity subset, then A/B against the matrix-core sums (one session,
# alternated), C5 and C3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "view_set_vs_oracle or second_colors or two_color or c5_sugar or sugar_normal" > gpurun_out/hits_tests.log 2>&1 || exit 1
OUTF=gpurun_out/hits_ab.txt
: > $OUTF
for round in 1 2; do
for WL in sugar c3; do
for S in hits mfma; do
  GSR_BWD_SUMS=$S timeout -k 10 200 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/hab_${WL}_${S}_${round}.json 2> gpurun_out/hab_${WL}_${S}_${round}.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hab_${WL}_${S}_${round}.json')); print('$WL', '$S', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
done
echo done
