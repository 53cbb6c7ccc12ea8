#!/bin/bash
# Round 5: the exchange serving path at N = 1, depth 4 / 6 / 7, a2a vs d2h results.
set -o pipefail
O=gpurun_out/r5ad
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
for d in 4 6 7; do
  for m in a2a d2h; do
    IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=$m step spmd_${m}_d$d 400 python bench.py --steps 20 --warmup 5 --depth $d --json-out $R/$O/spmd_${m}_d$d.json
  done
done
