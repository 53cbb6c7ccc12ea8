#!/bin/bash
# Round 5 (experiment): exchange path at N = 1 with in-order slots vs any free slot.
set -o pipefail
O=gpurun_out/r5ao
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
export IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h
step inorder 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/inorder.json
IGP_ANY_SLOT=1 step any 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/any.json
IGP_ANY_SLOT=1 step any_d7 300 python bench.py --steps 40 --warmup 5 --depth 7 --json-out $R/$O/any_d7.json
