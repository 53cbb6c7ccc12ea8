#!/bin/bash
# Round 6: PMC of the cfg3 device step at HEAD (tree_head after the LDS-traversal rework, K1,
# dedup insert, update): three passes within the per-block counter limits, engine_only cfg3,
# plus an unprofiled kernel-trace pass for the kernel times.
set -o pipefail
O=gpurun_out/r6aa
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
p=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
         "FETCH_SIZE SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
         "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_VMEM_WR"; do
  p=$((p+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $R/$O/pmc$p -o run -- \
    python $R/bench.py --scope engine_only --steps 40 --warmup 10 > $R/$O/pmc$p.log 2>&1
  rc=$?; echo "pmc$p rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- \
  python $R/bench.py --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/eng_kt.json > $R/$O/kt.log 2>&1
rc=$?; echo "kt rc=$rc" >> $R/$O/status.txt
