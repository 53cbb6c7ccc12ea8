#!/bin/bash
# Round 5: K1 PMC (SQ instruction / wait mix) on cold rotating batches, full kernel vs every
# account load and store skipped (AssembleArgs.ablate = 255), plus the counter list of the box.
set -o pipefail
O=gpurun_out/r5d
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/$O/counters.txt 2>&1; echo "list rc=$?" >> $R/$O/status.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for abl in 0 255; do
  for p in 1 2; do
    eval C=\$P$p
    KB_K1_MODES=- KB_ABLATE=$abl timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/$O/pmc_a${abl}_p$p -o run -- \
      python $R/tools/kbench.py --cold --rounds 1 --only dedup_insert > $R/$O/pmc_a${abl}_p$p.log 2>&1
    rc=$?; echo "pmc a$abl p$p rc=$rc" >> $R/$O/status.txt
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
