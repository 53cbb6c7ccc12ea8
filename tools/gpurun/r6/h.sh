#!/bin/bash
# Round 6: abuse steps without the split GRU clusters (default): cfg5 serving, mixed traffic.
set -o pipefail
O=gpurun_out/r6h
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
step tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_acct_gpu.py -p no:cacheprovider
step cfg5_t1 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1.json
step cfg5_t8 300 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg5_t8.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
step mixed_open_cap512 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --abuse-max-batch 512 --json-out $R/$O/mixed_open_cap512.json
step tree_bench 200 python tools/tree_bench.py
