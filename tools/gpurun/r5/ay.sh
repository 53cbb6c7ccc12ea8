#!/bin/bash
# Round 5: serving A/B, SSSE3 vs table decode of the UUID account key (AccountIndex::encode_key).
set -o pipefail
O=gpurun_out/r5ay
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
for i in 1 2 3 4; do
  step simd_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/simd_$i.json
  IGP_AB_SCALAR_KEY=1 step scalar_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/scalar_$i.json
done
