# Round-4 session d: hit-list tile backward with two waves per tile (k_render_bwd_tw<·, 2>) vs one; the
# bitwise kernel tests; bench A/B; counters of the default C3 build (lockstep matrix-core backward) and of C5.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -k "bitwise" > gpurun_out/${T}_bitwise.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 1
GSR_BWD_TW_WAVES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_bench_tw1.json 2> gpurun_out/${T}_bench_tw1.log || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --per-view-views 0 --extra-lines c5 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.log || exit 1
GSR_GAUSS_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-knn --extra-lines c5 > gpurun_out/${T}_bench_split.json 2> gpurun_out/${T}_bench_split.log || exit 1
# timing only: the C5 forward without the second colour's gathers (GSR_EXP_NOCOL2 diagnostic library)
for lib in product exp; do
  if [ $lib = exp ]; then export GSR_HIP_LIB=$PWD/threestudio-3dgs_amd/csrc/build_exp_NOCOL2/libgsr_hip_exp.so; fi
  timeout -k 10 300 python -u bench.py --workload sugar --steps 5 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 > gpurun_out/${T}_nocol2_$lib.json 2> gpurun_out/${T}_nocol2_$lib.log || exit 1
done
unset GSR_HIP_LIB
bash profiles/run_profiles.sh ${T} || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
