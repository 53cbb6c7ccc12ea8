#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench_drv.log 2>&1 || exit 3
IGP_NATIVE_DRIVER=0 timeout -k 10 300 python bench.py > gpurun_out/bench_py.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_drv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_drv -o run -- python $R/bench.py --steps 100 --warmup 10 > $R/gpurun_out/prof_drv.log 2>&1 || exit 6
