#!/bin/bash
# Round-6 session r: H28 (HEAD 285f60d) vs VG (k_view_grad loads its 16 items' reach words together before testing
# them, and stores the unreached items' zero means2D gradients after every test: one memory wait in its first
# pass instead of one per item), headline and 8-view sets alternated.
set -o pipefail
mkdir -p gpurun_out
BASE="--no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none"
for round in 1 2; do
  for spec in H28=build_ab/libgsr_hip_H28.so VG=build_ab/libgsr_hip_VG.so; do
    name=${spec%%=*}; lib=${spec#*=}
    for wl in "v64:--steps 10 --warmup 3" "v8:--views 8 --steps 30 --warmup 5"; do
      tag=${wl%%:*}; args=${wl#*:}
      GSR_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $BASE $args > gpurun_out/r06r_${tag}_${name}_${round}.json \
        2> gpurun_out/r06r_${tag}_${name}_${round}.log || exit 1
      python scripts/bench_summary.py gpurun_out/r06r_${tag}_${name}_${round}.json
    done
  done
done
echo "r06r ab done"
# kernel trace of the per-view drop-in path on the in-tree (HEAD) build: one step = 64 GaussianRasterizer calls
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06r_pv -o pv -- python3 bench.py --path per-view \
  --steps 1 --warmup 1 --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/prof_r06r_pv.log 2>&1 || exit 1
echo "r06r pv done"
