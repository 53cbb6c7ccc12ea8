#!/bin/bash
# round 3, pass n: PMC counters of the cfg4 chain kernels (pair-cluster vs one-workgroup 64-row):
# L2 hit / miss, MFMA busy, wave waits
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pr in 1 0; do
  IGP_MLP_PAIR=$pr timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/pmc$pr -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --numerics bf16 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/pmc$pr.log 2>&1 || exit 3
  python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmc$pr > $GRAFT_REPO_ROOT/$O/pmc_pair$pr.txt 2>&1 || exit 4
  IGP_MLP_PAIR=$pr timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pmcb$pr -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg4 --numerics bf16 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/pmcb$pr.log 2>&1 || exit 5
  python $GRAFT_REPO_ROOT/tools/pmc_summary.py /tmp/pmcb$pr > $GRAFT_REPO_ROOT/$O/pmcb_pair$pr.txt 2>&1 || exit 6
done
