#!/bin/bash
# Round 6: mixed traffic x4 with stall windows (where the intermittent tail comes from: which
# path, when, how long).
set -o pipefail
O=gpurun_out/r6aj
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
for i in 1 2 3 4; do
  step mixed_$i 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_$i.json
done
