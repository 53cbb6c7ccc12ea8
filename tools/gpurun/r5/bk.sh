#!/bin/bash
# Round 5: CU masks again with 2 tree groups (engine_only).
set -o pipefail
O=gpurun_out/r5bk
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
  for cs in none lo:192 lo:224 half; do
    n=$(echo $cs | tr ':' '_')
    IGP_CU_SPLIT=$cs step eng_${n}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_${n}_$i.json
  done
done
