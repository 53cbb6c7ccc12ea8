#!/bin/bash
# Round 6: cfg2 serving (1024-transaction requests) at depth 4 vs 6, interleaved, 3 runs each.
set -o pipefail
O=gpurun_out/r6ap
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
for i in 1 2 3; do
  for d in 4 6; do
    step cfg2_d${d}_$i 300 python bench.py --config cfg2 --steps 20 --warmup 5 --depth $d --json-out $R/$O/cfg2_d${d}_$i.json
  done
done
