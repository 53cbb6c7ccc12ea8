#!/bin/bash
# New GPU tests (velocity / batched features), then capacity A/B: cfg3 at 1 M vs 16 M accounts
# per GPU (same box): bench, K1 alone (kbench), K1 under overlap (kernel trace), K1 HBM reads (PMC)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2cap
O=gpurun_out/r2cap
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "watchdog or velocity" -x -v --timeout 120 --timeout-method thread > $O/t_gpu2.log 2>&1 || exit 1
for A in 1048576 16777216; do
  timeout -k 10 400 python bench.py --accounts $A --steps 300 --warmup 30 --json-out $O/bench_cfg3_acc$A.json > $O/bench_acc$A.log 2>&1 || exit 2
  timeout -k 10 400 python tools/kbench.py --accounts $A --rounds 30 --only feature_assemble_no_update,feature_assemble+single_update,full_step_graph --out $O/kbench_acc$A.json > $O/kbench_acc$A.log 2>&1 || exit 3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/cap$A -o run -- python bench.py --accounts $A --steps 100 --warmup 10 > $O/prof_acc$A.log 2>&1
  python tools/rocpd_stats.py /tmp/cap$A/run_results.db > $O/kernel_stats_acc$A.txt
  timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "feature_assemble" --output-format csv -d /tmp/pmc$A -o run -- python bench.py --accounts $A --steps 30 --warmup 5 > $O/pmc_acc$A.log 2>&1 || exit 4
  python tools/pmc_summary.py /tmp/pmc$A --batch 8192 > $O/pmc_k1_acc$A.txt
done
