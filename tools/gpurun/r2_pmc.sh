#!/bin/bash
# K1 alone at 64 K accounts (store inside the caches' reach), then K1 HBM reads per batch
# (TCC_EA0_RDREQ, PMC) at 1 M and 16 M accounts. IGP_ROCTX=0 tests whether the exit-time
# segfault under rocprofv3 comes from the roctx library the driver dlopens.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2cap
mkdir -p $O
timeout -k 10 300 python tools/kbench.py --accounts 65536 --rounds 30 --only feature_assemble_no_update,feature_assemble+single_update,full_step_graph --out $O/kbench_acc65536.json > $O/kbench_acc65536.log 2>&1 || exit 1
for A in 1048576 16777216; do
  IGP_ROCTX=0 timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "feature_assemble" --output-format csv -d /tmp/pmc$A -o run -- python bench.py --accounts $A --steps 30 --warmup 5 > $O/pmc_acc$A.log 2>&1
  rc=$?
  python tools/pmc_summary.py /tmp/pmc$A --batch 8192 > $O/pmc_k1_acc$A.txt
  [ $rc -eq 0 ] || exit 10
done
