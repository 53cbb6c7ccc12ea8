#!/bin/bash
# Round 6: serve depth 6 with the unary in-flight cap (4 while unary calls arrive): mixed
# traffic x3 at the defaults, the driver's serving command x2, engine tests.
set -o pipefail
O=gpurun_out/r6ah
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
step tests 500 python -u -m pytest tests/test_engine_gpu.py tests/test_acct_gpu.py -x -v --timeout 150 --timeout-method thread
for i in 1 2 3; do
  step mixed_$i 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_$i.json
done
for i in 1 2; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
done
