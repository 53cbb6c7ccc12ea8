#!/bin/bash
# Round 5: serving core slot-cycle breakdown, plain vs exchange path at N = 1.
set -o pipefail
O=gpurun_out/r5an
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
step plain 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/plain.json
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h step x_d2h 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/x_d2h.json
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h step x_d2h_d7 300 python bench.py --steps 40 --warmup 5 --depth 7 --json-out $R/$O/x_d2h_d7.json
