# Work-ordered tile dispatch: parity suite, then A/B against raster order (GSR_TILE_ORDER=raster) at 64 / 8
# views per launch, the per-view path and C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/order_parity.log 2>&1
echo "pytest exit $?" >> gpurun_out/order_parity.log
OUTF=gpurun_out/order_ab.txt
: > $OUTF
for rep in 1 2; do
for o in ordered raster; do
  if [ $o = raster ]; then export GSR_TILE_ORDER=raster; else unset GSR_TILE_ORDER; fi
  for args in "--views 64" "--views 8" "--path per-view --views 16" "--workload sugar"; do
    timeout -k 10 200 python -u bench.py $args --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/ord.json 2> gpurun_out/ord.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ord.json')); print('$o', '$args', d['value'], {a: b['ms_per_view'] for a, b in d['kernels'].items()})" >> $OUTF
  done
done
done
