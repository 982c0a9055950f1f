# One-view per-Gaussian backward (k_gauss_accum1): bitwise test, then the per-view drop-in path A/B
# (GSR_GAUSS_ACCUM1=0: the general kernel), one session, alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "one_view_gauss or view_set_vs_oracle or backward_is_repeatable" > gpurun_out/accum1_tests.log 2>&1 || exit 1
OUTF=gpurun_out/accum1_ab.txt
: > $OUTF
for round in 1 2; do
for A in 1 0; do
  GSR_GAUSS_ACCUM1=$A timeout -k 10 200 python -u bench.py --path per-view --views 16 --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/a1_$A.json 2> gpurun_out/a1_$A.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/a1_$A.json')); print('per-view', 'accum1=$A', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
