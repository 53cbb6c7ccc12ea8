#!/bin/bash
# N=2 rehearsal at HEAD on one GPU: two gloo ranks sharing the card (RCCL refuses two ranks on
# one device, so the exchange falls back to replicas together); checks the N>1 code path runs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dp2
mkdir -p $O
export IGP_DIST_BACKEND=gloo IGP_XCHG_INIT_S=60
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 60 --warmup 10 --accounts 262144 --json-out $O/bench_dp2.json > $O/bench_dp2.log 2>&1
echo "rc=$?" >> $O/bench_dp2.log
