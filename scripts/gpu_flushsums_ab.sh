# Hit-list backward: per-pair sums formed by the flush threads (no separate pass, one barrier less per batch)
# vs the separate batch-end pass (build_exp_PREV); C5 parity subset first, then one session alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "view_set_vs_oracle or second_colors or two_color or c5_sugar or sugar_normal" > gpurun_out/fs_tests.log 2>&1 || exit 1
OUTF=gpurun_out/flushsums_ab.txt
: > $OUTF
P=threestudio-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so
for round in 1 2; do
for spec in "merged $P" "prev threestudio-3dgs_amd/csrc/build_exp_PREV/libgsr_hip.so"; do
  set -- $spec
  GSR_HIP_LIB=$PWD/$2 timeout -k 10 200 python -u bench.py --workload sugar --steps 3 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/fs_$1.json 2> gpurun_out/fs_$1.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fs_$1.json')); print('sugar', '$1', $round, d['value'], {k: v['ms_per_view'] for k, v in d['kernels'].items()})" >> $OUTF
done
done
echo done
