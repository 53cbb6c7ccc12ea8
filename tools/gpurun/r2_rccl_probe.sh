#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 60 python tools/probe/rccl_order_probe.py > gpurun_out/r2/rccl_probe.log 2>&1 || exit 1
NCCL_LAUNCH_ORDER_IMPLICIT=0 timeout -k 10 60 python tools/probe/rccl_order_probe.py > gpurun_out/r2/rccl_probe_loi0.log 2>&1 || exit 2
NCCL_DEBUG=VERSION timeout -k 10 60 python -c "import torch; print(torch.cuda.nccl.version())" > gpurun_out/r2/rccl_version.log 2>&1 || exit 3
