#!/bin/bash
# Round 5: K1 kernel time vs batch rows (2048 / 4096 / 8192 / 16384), full and every account
# access skipped: does K1's time scale with the number of waves (a serialized resource)?
set -o pipefail
O=gpurun_out/r5i
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
for b in 2048 4096 8192 16384; do
  KB_K1_MODES=- KB_ABLATE=0,255 timeout -k 10 300 python tools/kbench.py --cold --rounds 2 --batch $b --only dedup_insert > $R/$O/kbench_$b.log 2>&1
  rc=$?; echo "kbench $b rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
