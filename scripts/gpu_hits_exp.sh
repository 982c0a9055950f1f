# Hit-list backward: where C5's backward blend time goes (GSR_EXP_* builds, timing only; their gradients are
# wrong), one session, builds alternated.
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/hits_exp.txt
: > $OUTF
for round in 1; do
for v in base NOGROUP NOREACH; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/hx_$v.json 2> gpurun_out/hx_$v.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hx_$v.json')); print('sugar', '$v', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
