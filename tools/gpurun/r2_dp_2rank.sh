#!/bin/bash
# exchange kernels with N>1 layouts; 2 ranks sharing one GPU (RCCL refuses -> replicas fallback)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/t_dp.log 2>&1 || exit 1
export IGP_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 60 --warmup 10 --accounts 262144 > gpurun_out/r2/bench_dp2_shared.log 2>&1
echo "rc=$?" >> gpurun_out/r2/bench_dp2_shared.log
