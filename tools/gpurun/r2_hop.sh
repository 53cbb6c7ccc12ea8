#!/bin/bash
# cross-queue hand-off cost probe (tools/probe/queue_hop_probe.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2hop
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 ./tools/probe/queue_hop_probe 400 > gpurun_out/r2hop/hop.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 ./tools/probe/queue_hop_probe 1000 >> gpurun_out/r2hop/hop.log 2>&1 || exit 2
