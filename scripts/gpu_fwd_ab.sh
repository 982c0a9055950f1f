set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -rf -k "forward_kernels or c1 or ragged or flat or culling" --timeout 300 --timeout-method thread > gpurun_out/r02_fwdtile_tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/r02_fwdtile_tests.log
: > gpurun_out/r02_fwd_ab.txt
for k in tile quadrant tile quadrant; do
  GSR_FWD_KERNEL=$k timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/fwd_$k.json 2> gpurun_out/fwd_$k.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fwd_$k.json')); print('$k', d['value'], {k2: v['ms_per_view'] for k2, v in d['kernels'].items()})" >> gpurun_out/r02_fwd_ab.txt
  GSR_FWD_KERNEL=$k timeout -k 10 200 python -u bench.py --workload sugar --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/fwds_$k.json 2> gpurun_out/fwds_$k.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fwds_$k.json')); print('sugar $k', d['value'], {k2: v['ms_per_view'] for k2, v in d['kernels'].items()})" >> gpurun_out/r02_fwd_ab.txt
done
