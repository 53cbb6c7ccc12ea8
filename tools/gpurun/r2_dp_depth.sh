#!/bin/bash
# exchange at world 1: RCCL captured into the graphs vs issued by the driver
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t_dp.log 2>&1 || exit 1
IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/r2/bench_xchg1_cap.log 2>&1 || exit 2
IGP_XCHG_CAPTURE=0 IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/r2/bench_xchg1_nocap.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/r2/bench_plain.log 2>&1 || exit 4
