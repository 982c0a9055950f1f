# Dispatch-order chunk size sweep (views interleaved per chunk): product (8) vs build_exp_CH{1,4,16}
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/chunk.txt
: > $OUTF
for rep in 1 2; do
for v in base CH1 CH4 CH16; do
  if [ $v = base ]; then lib=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so; else lib=threestudio-3dgs_amd/csrc/build_exp_$v/libgsr_hip.so; fi
  for a in "--views 64" "--views 8" "--workload sugar"; do
    GSR_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py $a --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/ch.json 2> gpurun_out/ch.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ch.json')); print('$v', '$a', d['value'], {x: y['ms_per_view'] for x, y in d['kernels'].items() if x.startswith('render')})" >> $OUTF
  done
done
done
