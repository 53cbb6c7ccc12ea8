#!/bin/bash
# Round 5: cfg4 engine_only, split-chain rows per workgroup 64 (default) vs 32.
set -o pipefail
O=gpurun_out/r5bm
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
for i in 1 2; do
  for r in 64 32; do
    IGP_MLP_SPLIT_ROWS=$r step cfg4_r${r}_$i 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_r${r}_$i.json
  done
done
