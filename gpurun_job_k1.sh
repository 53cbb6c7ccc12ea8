#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k1_tests.log 2>&1 || exit 3
timeout -k 10 200 python tools/kbench.py --rounds 50 > gpurun_out/kb_k1.log 2>&1 || exit 4
timeout -k 10 200 python bench.py --steps 300 --warmup 50 > gpurun_out/k1_bench.log 2>&1 || exit 5
