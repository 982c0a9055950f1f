# Host-gap check: the same bench with and without the per-stage HIP-event profile, alternated (timing only).
set -o pipefail
mkdir -p gpurun_out
OUTF=gpurun_out/r02_hostgap.txt
: > $OUTF
for v in prof noprof prof noprof; do
  flag=""; [ $v = noprof ] && flag="--no-profile"
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-knn --per-view-views 0 $flag > gpurun_out/hg_$v.json 2> gpurun_out/hg_$v.log || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/hg_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" >> $OUTF
done
