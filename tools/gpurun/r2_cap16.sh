#!/bin/bash
# General-tree GPU tests, then cfg3 at 16 M accounts per GPU: bench, K1 alone (kbench), and K1
# under overlap (kernel trace; the last GPU step: rocprofv3 can segfault at process exit)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2cap
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_trees_general_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t_trees_gpu.log 2>&1 || exit 1
A=16777216
timeout -k 10 500 python bench.py --accounts $A --steps 300 --warmup 30 --json-out $O/bench_cfg3_acc$A.json > $O/bench_acc$A.log 2>&1 || exit 2
timeout -k 10 500 python tools/kbench.py --accounts $A --rounds 30 --only feature_assemble_no_update,feature_assemble+single_update,full_step_graph --out $O/kbench_acc$A.json > $O/kbench_acc$A.log 2>&1 || exit 3
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/cap$A -o run -- python bench.py --accounts $A --steps 100 --warmup 10 > $O/prof_acc$A.log 2>&1
python tools/rocpd_stats.py /tmp/cap$A/run_results.db > $O/kernel_stats_acc$A.txt
