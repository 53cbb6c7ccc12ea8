#!/bin/bash
# Round 6: account FIFO as a vector swapped whole into the step under the lock (B) vs a deque (A):
# cfg4 and cfg5 through the router, interleaved.
set -o pipefail
O=gpurun_out/r6aq
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
N=$R/igaming_platform_amd/_native.cpython-310-x86_64-linux-gnu.so
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2 3; do
  for v in A B; do
    cp $R/ab/_native_$v.so $N
    IGP_BENCH_THREADS_OUT=$R/$O/cfg4_${v}${i}_threads.json step cfg4_${v}$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_${v}$i.json
  done
done
for v in A B; do
  cp $R/ab/_native_$v.so $N
  step cfg5_$v 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_$v.json
done
cp $R/ab/_native_B.so $N
