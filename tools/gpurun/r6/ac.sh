#!/bin/bash
# Round 6: the multi-rank serving path on real GPU processes (first time): world 2 and world 4
# with every rank on the box's one GPU (node-shared rows / results regions: no RCCL
# communicator, so ranks may share a device); SPMD world 1 with the exchange wait accounting;
# cfg5 through the account routers at world 2 (the /dev/shm owner mailbox).
set -o pipefail
O=gpurun_out/r6ac
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
IGP_BENCH_SPMD=1 step spmd1 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd1.json
step w2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --threads 8 --json-out $R/$O/w2.json
step w4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 10 --warmup 3 --threads 4 --json-out $R/$O/w4.json
step cfg5_w2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --config cfg5 --steps 3 --warmup 1 --json-out $R/$O/cfg5_w2.json
