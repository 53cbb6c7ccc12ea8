#!/bin/bash
# Round 5: K1 latencies from the derived SQ level counters (VMEM / SMEM / LDS / instruction fetch)
set -o pipefail
O=gpurun_out/r5j
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
i=0
for abl in 0 255; do
  for C in "VmemLatency SmemLatency" "InstrFetchLatency LdsLatency" "MeanOccupancyPerActiveCU"; do
    i=$((i+1))
    KB_K1_MODES=- KB_ABLATE=$abl timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/$O/pmc_a${abl}_$i -o run -- \
      python $R/tools/kbench.py --cold --rounds 1 --only dedup_insert > $R/$O/pmc_a${abl}_$i.log 2>&1
    rc=$?; echo "pmc a$abl $i rc=$rc" >> $R/$O/status.txt
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
