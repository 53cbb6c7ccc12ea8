#!/bin/bash
# Round 6: account core releases a device slot once its outputs are copied out (answers written
# from the copy): account GPU tests, cfg5 x3, cfg4 x2, mixed traffic.
set -o pipefail
O=gpurun_out/r6w
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
step tests 400 python -u -m pytest tests/test_acct_gpu.py -x -v --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step cfg5_$i 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_$i.json
done
for i in 1 2; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg4_${i}_threads.json step cfg4_$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_$i.json
done
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
