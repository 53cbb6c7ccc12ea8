#!/bin/bash
# Round 5: exchange serving path at N = 1: CU split A/B (none vs half) and a kernel trace.
set -o pipefail
O=gpurun_out/r5ai
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
for i in 1 2; do
  for cs in none half; do
    IGP_CU_SPLIT=$cs step cu_${cs}_$i 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/cu_${cs}_$i.json
  done
done
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/bench.py --steps 4 --warmup 2 --json-out $R/$O/prof.json
