#!/bin/bash
# GPU session: rehearse the N = 2 bench path on a one-GPU box (two ranks sharing the GPU over gloo).
mkdir -p gpurun_out
TAG=${1:-rehearse2}
for g in overlap sync; do
  GSR_BENCH_BACKEND=gloo GSR_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-knn \
    --per-view-views 0 --views 16 --gather $g > gpurun_out/${TAG}_${g}.json 2> gpurun_out/${TAG}_${g}.log || exit $?
  python scripts/bench_summary.py gpurun_out/${TAG}_${g}.json
done
echo done
