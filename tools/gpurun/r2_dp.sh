#!/bin/bash
# owner-routed RCCL exchange on one GPU (world 1): numerics vs the plain pipeline, SPMD engine,
# exchange bench vs the plain bench (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/t_dp.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r2/bench_cfg3_plain.log 2>&1 || exit 2
IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/r2/bench_cfg3_xchg1.log 2>&1 || exit 3
