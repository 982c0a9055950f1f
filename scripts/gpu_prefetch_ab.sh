# Backward-blend staging prefetch depth: record pieces two batches ahead (product for the two-colour backward)
# vs one (GSR_PREFETCH1 build); the one-colour backward with two (GSR_PREFETCH2_ALL build) vs one (product).
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/prefetch_ab.txt
: > $OUTF
P=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so
for round in 1 2; do
for spec in "sugar product $P" "sugar p1 threestudio-3dgs_amd/csrc/build_exp_P1/libgsr_hip.so" "c3 product $P" "c3 p2all threestudio-3dgs_amd/csrc/build_exp_P2ALL/libgsr_hip.so"; do
  set -- $spec
  GSR_HIP_LIB=$PWD/$3 timeout -k 10 200 python -u bench.py --workload $1 --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/pf_$1_$2.json 2> gpurun_out/pf_$1_$2.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pf_$1_$2.json')); print('$1', '$2', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
