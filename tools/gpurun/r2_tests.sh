#!/bin/bash
# full GPU suite at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/head
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/head/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --json-out gpurun_out/head/bench_cfg3.json > gpurun_out/head/bench.log 2>&1 || exit 2
