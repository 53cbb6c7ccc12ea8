#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_kb
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_kb -o run -- python $R/tools/kbench.py --rounds 20 > $R/gpurun_out/prof_kb.log 2>&1 || exit 3
