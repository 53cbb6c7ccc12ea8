#!/bin/bash
# K1 HBM reads per batch at 16 M accounts (PMC); exit-time segfault under rocprofv3 checks:
# the PMC run without CU-masked streams (IGP_CU_SPLIT=none), then a kernel-trace run with them
# (now destroyed at interpreter exit) as the last GPU step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2cap
mkdir -p $O
A=16777216
IGP_CU_SPLIT=none timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "feature_assemble" --output-format csv -d /tmp/pmc$A -o run -- python bench.py --accounts $A --steps 30 --warmup 5 > $O/pmc_acc$A.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/pmc$A --batch 8192 > $O/pmc_k1_acc$A.txt
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof3 -o run -- python bench.py --steps 100 --warmup 10 > $O/prof_atexit.log 2>&1
rc=$?
python tools/rocpd_stats.py /tmp/prof3/run_results.db > $O/kernel_stats_atexit.txt
exit $rc
