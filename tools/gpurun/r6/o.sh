#!/bin/bash
# Round 6: account-router benches with batched submitters (1 / 4 / 8 threads, default depths);
# mixed traffic.
set -o pipefail
O=gpurun_out/r6o
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
for c in cfg5 cfg4; do
  for t in 1 4 8; do
    step ${c}_t$t 300 python bench.py --config $c --steps 5 --warmup 1 --drive-threads $t --json-out $R/$O/${c}_t$t.json
  done
done
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
