#!/bin/bash
# Round 5: serving A/B tree groups 2 vs 4 (interleaved, 5 pairs).
set -o pipefail
O=gpurun_out/r5bg
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2 3 4 5; do
  for g in 2 4; do
    IGP_TREE_GROUPS=$g step srv_g${g}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_g${g}_$i.json
  done
done
