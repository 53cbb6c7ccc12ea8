#!/bin/bash
# Round 6: mixed traffic after the link-index reader hand-over and the 200 us link wait;
# abuse device depth 2 / 3.
set -o pipefail
O=gpurun_out/r6p
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
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
step mixed_d3 400 python tools/bench_mixed.py --seconds 5 --acct-depth 3 --json-out $R/$O/mixed_d3.json
step mixed_open_d3 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --acct-depth 3 --json-out $R/$O/mixed_open_d3.json
