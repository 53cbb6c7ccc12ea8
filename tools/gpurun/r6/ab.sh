#!/bin/bash
# Round 6: account answers with batched sink counters and the LTV timestamp written in place:
# cfg4 x3, cfg5; mixed traffic x3; serving x2.
set -o pipefail
O=gpurun_out/r6ab
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
  IGP_BENCH_THREADS_OUT=$R/$O/cfg4_${i}_threads.json step cfg4_$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_$i.json
done
step cfg5 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5.json
for i in 1 2; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
done
for i in 1 2 3; do
  step mixed_$i 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_$i.json
done
