#!/bin/bash
# Round 5: per-thread host CPU of the plain vs exchange serving path at N = 1 (IGP_BENCH_THREADS_OUT).
set -o pipefail
O=gpurun_out/r5ah
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
IGP_BENCH_THREADS_OUT=$R/$O/threads_plain.json step thr_plain 300 python bench.py --steps 60 --warmup 5 --json-out $R/$O/thr_plain.json
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h IGP_BENCH_THREADS_OUT=$R/$O/threads_spmd.json step thr_spmd 300 python bench.py --steps 60 --warmup 5 --json-out $R/$O/thr_spmd.json
