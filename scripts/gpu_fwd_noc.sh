# Timing only: the C5 quadrant-wave forward without the records' colour field loads (GSR_EXP_FWD_NOC build;
# wrong colours) vs the product, and its FETCH_SIZE — is the forward's HBM traffic the per-wave record gathers?
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/fwd_noc.txt
: > $OUTF
P=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so
for round in 1 2; do
for spec in "product $P" "noc threestudio-3dgs_amd/csrc/build_exp_FWDNOC/libgsr_hip.so"; do
  set -- $spec
  GSR_HIP_LIB=$PWD/$2 timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/fn_$1.json 2> gpurun_out/fn_$1.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fn_$1.json')); print('sugar', '$1', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_FWDNOC/libgsr_hip.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fwdnoc/fetch -o run --output-format csv -- python3 bench.py --workload sugar --steps 2 --warmup 1 --no-cpu-baseline --per-view-views 0 --no-knn --no-profile > gpurun_out/prof_fwdnoc.log 2>&1 || exit 1
echo done
