#!/bin/bash
# Round 5: account-router bench submit threads A/B (cfg5 / cfg4, interleaved).
set -o pipefail
O=gpurun_out/r5bj
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
  for t in 1 2 4; do
    step cfg5_t${t}_$i 300 python bench.py --config cfg5 --steps 20 --warmup 5 --drive-threads $t --json-out $R/$O/cfg5_t${t}_$i.json
  done
  for t in 1 2; do
    step cfg4_t${t}_$i 300 python bench.py --config cfg4 --steps 20 --warmup 5 --drive-threads $t --json-out $R/$O/cfg4_t${t}_$i.json
  done
done
