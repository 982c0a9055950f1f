# Where the backward blend's time goes now (GSR_EXP_* builds, timing only), C5 and C3, one session.
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/r03d_exp.txt
: > $OUTF
for WL in sugar c3; do
for v in base NOMFMA NOGROUP NOFLUSH; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.log || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/exp_$v.json')); print('$WL', '$v', d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
