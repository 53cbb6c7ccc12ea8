#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_x
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_x -o run -- python $R/tools/kbench.py --rounds 3 --only h2d_slab > $R/gpurun_out/kb_x.log 2>&1 || exit 3
