#!/bin/bash
# Round 5: exchange serving path at N = 1: pipeline depth A/B (CU split none).
set -o pipefail
O=gpurun_out/r5aj
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
export IGP_XCHG_RESULTS=d2h IGP_CU_SPLIT=none
for i in 1 2; do
  for d in 4 6 7; do
    IGP_BENCH_SPMD=1 step x_d${d}_$i 300 python bench.py --steps 40 --warmup 5 --depth $d --json-out $R/$O/x_d${d}_$i.json
  done
done
unset IGP_CU_SPLIT
for d in 4 6; do
  step p_d${d} 300 python bench.py --steps 40 --warmup 5 --depth $d --json-out $R/$O/p_d${d}.json
done
