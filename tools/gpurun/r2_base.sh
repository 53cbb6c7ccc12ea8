#!/bin/bash
# round 2 baseline at HEAD: GPU tests + cfg3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/t_gpu.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --json-out gpurun_out/r2/bench_cfg3.json > gpurun_out/r2/bench_cfg3.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --config cfg4 --json-out gpurun_out/r2/bench_cfg4.json > gpurun_out/r2/bench_cfg4.log 2>&1 || exit 3
