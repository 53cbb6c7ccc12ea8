#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k1_tests.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 300 --warmup 50 > gpurun_out/k1_bench.log 2>&1 || exit 5
cd /tmp
rm -rf $R/gpurun_out/prof_kb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kb -o run -- python $R/tools/kbench.py --rounds 20 > $R/gpurun_out/prof_kb.log 2>&1 || exit 4
