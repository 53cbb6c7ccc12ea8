#!/bin/bash
# one GPU round: tests, smoke, bench at several pipeline depths + kernel breakdown of the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/t_gpu_all.log 2>&1 || exit 1
for d in 2 3 4; do
  timeout -k 10 300 python bench.py --depth $d > gpurun_out/bench_cfg3_d$d.log 2>&1 || exit 3
done
timeout -k 10 300 python tools/kbench.py --rounds 40 > gpurun_out/kbench2.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3b -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/prof3b.log 2>&1 || exit 5
