#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_cfg3 $R/gpurun_out/prof_cfg5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg3 -o run -- python $R/bench.py --steps 100 --warmup 10 > $R/gpurun_out/prof_cfg3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg5 -o run -- python $R/bench.py --config cfg5 --steps 50 --warmup 5 > $R/gpurun_out/prof_cfg5.log 2>&1 || exit 2
