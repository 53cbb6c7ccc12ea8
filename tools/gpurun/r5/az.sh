#!/bin/bash
# Round 5: engine_only cfg3 pipeline depth A/B (4-7 batches in flight).
set -o pipefail
O=gpurun_out/r5az
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
  for d in 4 5 6 7; do
    step eng_d${d}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --depth $d --json-out $R/$O/eng_d${d}_$i.json
  done
done
