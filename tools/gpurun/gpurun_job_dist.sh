#!/bin/bash
# rehearse the multi-rank bench path on a 1-GPU box: 2 ranks share cuda:0 over gloo
set -o pipefail
mkdir -p gpurun_out
export IGP_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --accounts 262144 > gpurun_out/dist_cfg3.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config cfg5 --steps 10 --warmup 2 --accounts 65536 > gpurun_out/dist_cfg5.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --config cfg5 --steps 50 --warmup 5 > gpurun_out/cfg5.log 2>&1 || exit 3
