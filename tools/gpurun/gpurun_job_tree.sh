#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/tree_bench.py > gpurun_out/tree_sweep2.log 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tree_tests.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 300 --warmup 50 > gpurun_out/tree_bench.log 2>&1 || exit 5
