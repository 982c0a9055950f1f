# A/B of an experiment build against the product on one workload (alternated; timing only).
# usage: EXP=<build_exp_ suffix> WL=<c3|sugar> bash scripts/gpu_ab.sh, after (CPU side)
#   make -C threestudio-3dgs_amd/csrc OBJDIR=build_exp_<X> OUT=build_exp_<X>/libgsr_hip.so EXTRA=-DGSR_EXP_<X>
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/ab_${EXP}_${WL}.txt
: > $OUTF
for v in base $EXP base $EXP; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
