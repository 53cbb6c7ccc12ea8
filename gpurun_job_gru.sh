#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/gru_ws_trace.py 4096 > gpurun_out/gru_trace.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/cfg5.log 2>&1 || exit 3
timeout -k 10 300 python tools/gru_bench.py > gpurun_out/gru_bench.log 2>&1 || exit 4
