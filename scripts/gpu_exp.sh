# A/B of the backward blend's parts (GSR_EXP_* builds, timing only: their gradients are wrong)
set -o pipefail
mkdir -p gpurun_out
WL=${WL:-sugar}
OUTF=gpurun_out/r02_exp_${WL}.txt
: > $OUTF
for v in base NOREPLAY NOMFMA NOFLUSH NOCULL NOGROUP; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.log || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/exp_$v.json')); print('$v', d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
