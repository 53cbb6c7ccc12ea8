#!/bin/bash
# Round 5: exchange path (recorded state / model stages) at N = 1: pipeline depth A/B.
set -o pipefail
O=gpurun_out/r5am
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
export IGP_BENCH_SPMD=1
for i in 1 2; do
  for m in d2h a2a; do
    for d in 4 6 7; do
      IGP_XCHG_RESULTS=$m step x_${m}_d${d}_$i 300 python bench.py --steps 40 --warmup 5 --depth $d --json-out $R/$O/x_${m}_d${d}_$i.json
    done
  done
done
