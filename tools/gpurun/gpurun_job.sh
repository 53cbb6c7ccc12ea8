#!/bin/bash
# one GPU round: tests, smoke, headline bench, pipeline trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/t_gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench_cfg3.log 2>&1 || exit 3
timeout -k 10 300 python tools/overlap_probe.py > gpurun_out/overlap.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3c -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --rounds 20 > $GRAFT_REPO_ROOT/gpurun_out/prof3c.log 2>&1 || exit 5
