#!/bin/bash
# Round 6: account-router benches at the new defaults (4 drive threads, (depth + 3)-step window):
# cfg5 x3, cfg5 at 8 threads / a 32 k window, cfg4 x2.
set -o pipefail
O=gpurun_out/r6v
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
  step cfg5_$i 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_$i.json
done
step cfg5_t8 300 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg5_t8.json
step cfg5_w32k 300 python bench.py --config cfg5 --steps 5 --warmup 1 --inflight 32768 --json-out $R/$O/cfg5_w32k.json
for i in 1 2; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg4_${i}_threads.json step cfg4_$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_$i.json
done
