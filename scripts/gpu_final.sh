# Round-end GPU session: parity suite, profiles (kernel trace, FETCH/WRITE/VALU passes, pair counts), bench lines.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1
echo "pytest exit $?" >> gpurun_out/${TAG}_parity.log
bash profiles/run_profiles.sh $TAG || exit 1
# the bench lines below read this session's counters and pair counts (the box's copy of profiles/)
python profiles/summarize.py $TAG > gpurun_out/${TAG}_summarize.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/diag_pairs.py $TAG > gpurun_out/${TAG}_pairs.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/diag_pairs.py $TAG sugar > gpurun_out/${TAG}_pairs_sugar.log 2>&1 || exit 1
cp gpurun_out/pairs_${TAG}.json profiles/${TAG}_pairs.json && cp gpurun_out/pairs_${TAG}_sugar.json profiles/${TAG}_pairs_sugar.json
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit 1
timeout -k 10 400 python -u bench.py --workload sugar --no-cpu-baseline --no-knn > gpurun_out/${TAG}_bench_sugar.json 2> gpurun_out/${TAG}_bench_sugar.log || exit 1
timeout -k 10 400 python -u bench.py --epilogue shading --no-cpu-baseline --no-knn > gpurun_out/${TAG}_bench_shading.json 2> gpurun_out/${TAG}_bench_shading.log
