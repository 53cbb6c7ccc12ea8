#!/bin/bash
# Round 6: mixed traffic at scoring-pipeline depth 4 vs 6, interleaved, 3 runs each (the unary
# tails against the ScoreBatch throughput gain of depth 6).
set -o pipefail
O=gpurun_out/r6af
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
    step mixed_d${d}_$i 400 python tools/bench_mixed.py --seconds 5 --serve-depth $d --json-out $R/$O/mixed_d${d}_$i.json
  done
done
