#!/bin/bash
# 2 ranks sharing one GPU through the bench's N>1 path (RCCL refuses two ranks on one device ->
# the agreed replicas fallback): checks the communicator deadline / fallback logic end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2dp2
export IGP_DIST_BACKEND=gloo IGP_XCHG_INIT_S=60
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 60 --warmup 10 --accounts 262144 > gpurun_out/r2dp2/bench_dp2_shared.log 2>&1
echo "rc=$?" >> gpurun_out/r2dp2/bench_dp2_shared.log
