#!/bin/bash
# Round 6: tree traversal ILP A/B (4 / 8 / 16 traversals in flight per lane) on the cfg3
# tree_head kernel: engine_only and serving, plus the standalone tree bench; mixed traffic with
# the 500 us link wait.
set -o pipefail
O=gpurun_out/r6k
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
for ilp in 4 8 16; do
  step tree_$ilp 200 env IGP_TR_ILP=$ilp python tools/tree_bench.py
  step eng_$ilp 300 env IGP_TR_ILP=$ilp python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_$ilp.json
  step srv_$ilp 300 env IGP_TR_ILP=$ilp python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$ilp.json
done
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
