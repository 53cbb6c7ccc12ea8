#!/bin/bash
# Round 5: is K1 bound by instruction fetch? Instruction-cache counters of K1 (full / every account
# access skipped) and K1 launched twice back to back (1024: second launch with warm caches).
set -o pipefail
O=gpurun_out/r5g
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
KB_K1_MODES=- KB_ABLATE=255,1279,2,1026 timeout -k 10 300 python tools/kbench.py --cold --rounds 3 --only dedup_insert > $R/$O/kbench.log 2>&1
echo "kbench rc=$?" >> $R/$O/status.txt
cd /tmp
for abl in 0 255; do
  KB_K1_MODES=- KB_ABLATE=$abl timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $R/$O/pmc_a$abl -o run -- \
    python $R/tools/kbench.py --cold --rounds 1 --only dedup_insert > $R/$O/pmc_a$abl.log 2>&1
  rc=$?; echo "pmc a$abl rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
