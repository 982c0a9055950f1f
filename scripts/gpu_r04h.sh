# Round-4 session h: counters of the current kernels (C3 default and C5) for bench.py's roofline fields.
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04h}
bash profiles/run_profiles.sh ${T} || exit 1
bash profiles/run_profiles.sh ${T}_sugar --workload sugar || exit 1
echo "session $T done"
