# Packed replay steps in the hit-list backward: parity subset (incl. packed vs one-per-step bitwise), then
# A/B (one session, alternated): C5 packed / unpacked hits / matrix-core sums, C4-native 256^2 hits vs mfma.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "hit_list or view_set_vs_oracle or second_colors or two_color or c5_sugar or sugar_normal" > gpurun_out/pack_tests.log 2>&1 || exit 1
OUTF=gpurun_out/pack_ab.txt
: > $OUTF
for round in 1 2; do
for S in pack nopack mfma; do
  case $S in pack) E="GSR_BWD_SUMS=hits";; nopack) E="GSR_BWD_SUMS=hits GSR_BWD_PACK=0";; mfma) E="GSR_BWD_SUMS=mfma";; esac
  env $E timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/pk_sugar_$S.json 2> gpurun_out/pk_sugar_$S.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pk_sugar_$S.json')); print('sugar', '$S', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
for S in pack mfma; do
  case $S in pack) E="GSR_BWD_SUMS=hits";; mfma) E="GSR_BWD_SUMS=mfma";; esac
  env $E timeout -k 10 200 python -u bench.py --res 256 --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/pk_256_$S.json 2> gpurun_out/pk_256_$S.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pk_256_$S.json')); print('c3-256', '$S', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
