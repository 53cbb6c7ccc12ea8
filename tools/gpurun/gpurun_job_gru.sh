#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/gru_ws_trace.py 4096 > gpurun_out/gru_trace.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gru.log 2>&1 || exit 2
