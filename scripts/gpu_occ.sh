# Occupancy sensitivity of the backward blend (LDS padding: 5 -> 4 -> 3 workgroups per CU; timing only)
# and the per-tile quadrant-imbalance bound (diagnostic build).  Build first (CPU side):
#   for p in 8192 22000; do make -C threestudio-3dgs_amd/csrc OBJDIR=build_exp_PAD$p OUT=build_exp_PAD$p/libgsr_hip.so \
#     EXTRA=-DGSR_EXP_LDSPAD=$p; done; make -C threestudio-3dgs_amd/csrc diag
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/occ.txt
: > $OUTF
for v in base PAD8192 PAD22000 base; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/occ_$v.json 2> gpurun_out/occ_$v.log || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/occ_$v.json')); print('$v', d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
timeout -k 10 300 python -u profiles/diag_pairs.py occ > gpurun_out/occ_pairs.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/diag_pairs.py occ sugar > gpurun_out/occ_pairs_sugar.log 2>&1
