#!/bin/bash
# one GPU round: tests, smoke, rocprofv3 stats of the headline and the GRU config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/t_gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof5.log 2>&1 || exit 4
