# Round-4 session e: quadrant masks in the unpacked keys (span_quads per row in k_emit), one-wave tile backward by
# default (replay software-pipelined), fused per-Gaussian backward without SH only, branch-free full groups in the
# lockstep backward.  Full GPU suite, bench, masks A/B, C5 counters.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_TILE_KEYS=plain timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_plain.json 2> gpurun_out/${T}_c5_plain.log || exit 1
timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_c5_masks.json 2> gpurun_out/${T}_c5_masks.log || exit 1
# C3 backward: full groups of 8 replayed two steps per scheduling region (GSR_BWD_OVERLAP=2, 4 VGPRs spilled) vs one
GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_OVL2/libgsr_hip_exp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/${T}_ovl2.json 2> gpurun_out/${T}_ovl2.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines none > gpurun_out/${T}_ovl1.json 2> gpurun_out/${T}_ovl1.log || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
