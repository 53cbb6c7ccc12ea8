#!/bin/bash
# Round 5: tree groups per launch (waves per SIMD of tree_head) A/B, engine_only and serving.
set -o pipefail
O=gpurun_out/r5be
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
for i in 1 2; do
  for g in 4 8 12 2; do
    IGP_TREE_GROUPS=$g step eng_g${g}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_g${g}_$i.json
  done
done
for i in 1 2; do
  for g in 4 8; do
    IGP_TREE_GROUPS=$g step srv_g${g}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_g${g}_$i.json
  done
done
