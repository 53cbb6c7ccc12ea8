#!/bin/bash
# Round 6: cfg4 engine_only at depth 3 with 32-row vs 64-row split-chain tiles (32 rows run
# 93.5 vs 120 us alone, r6/z; round 5 measured 32 slower in the depth-4 pipeline), interleaved.
set -o pipefail
O=gpurun_out/r6ao
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
for i in 1 2 3; do
  for r in 64 32; do
    IGP_MLP_SPLIT_ROWS=$r step eng4_r${r}_$i 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/eng4_r${r}_$i.json
  done
done
for r in 64 32; do
  IGP_MLP_SPLIT_ROWS=$r step eng4_d2_r${r} 300 python bench.py --config cfg4 --scope engine_only --depth 2 --steps 200 --warmup 20 --json-out $R/$O/eng4_d2_r${r}.json
done
