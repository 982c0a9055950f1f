# Two-colour forward with one staged batch per tile: bitwise tests + C5 parity subset, then A/B vs the
# quadrant waves gathering on their own (GSR_FWD_SHARED=0), one session alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "forward_kernels_bitwise or second_colors or two_color or c5_sugar or sugar_normal" > gpurun_out/fsh_tests.log 2>&1 || exit 1
OUTF=gpurun_out/fwd_shared_ab.txt
: > $OUTF
for round in 1 2; do
for S in 1 0; do
  GSR_FWD_SHARED=$S timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/fsh_$S.json 2> gpurun_out/fsh_$S.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fsh_$S.json')); print('sugar', 'shared=$S', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
