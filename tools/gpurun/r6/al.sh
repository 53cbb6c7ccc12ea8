#!/bin/bash
# Round 6: tree groups per 8192-row launch after the LDS traversal rework (the group heuristic
# was tuned before it): 2 / 3 / 4 groups, engine_only and serving interleaved, 2 runs each.
set -o pipefail
O=gpurun_out/r6al
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
  for g in 2 3 4; do
    IGP_TREE_GROUPS=$g step eng_g${g}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_g${g}_$i.json
    IGP_TREE_GROUPS=$g step srv_g${g}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_g${g}_$i.json
  done
done
