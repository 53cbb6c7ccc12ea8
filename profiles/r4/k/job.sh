#!/bin/bash
# Round 4: K1 on cold (uniform) batches: kernel time and phase trace (tools/kbench.py --cold).
set -o pipefail
O=gpurun_out/r4k
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -12 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step k1_cold 300 python tools/kbench.py --cold --rounds 20 --only dedup_insert
step k1_hot 300 python tools/kbench.py --rounds 20 --only dedup_insert
