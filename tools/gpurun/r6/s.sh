#!/bin/bash
# Round 6: account-router slot cycle (submit / turn-around / free time per step, issue reasons)
# for cfg5 at 1 / 4 drive threads and cfg4 at 4.
set -o pipefail
O=gpurun_out/r6s
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
for t in 1 4; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg5_t${t}_threads.json step cfg5_t$t 300 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads $t --json-out $R/$O/cfg5_t$t.json
done
IGP_BENCH_THREADS_OUT=$R/$O/cfg4_t4_threads.json step cfg4_t4 300 python bench.py --config cfg4 --steps 5 --warmup 1 --drive-threads 4 --json-out $R/$O/cfg4_t4.json
