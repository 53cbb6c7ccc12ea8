#!/bin/bash
# Round 5: serving A/B, AccountIndex probe prefetch distance (rows ahead) 16 / 32 / 64.
set -o pipefail
O=gpurun_out/r5ax
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
  for k in 16 32 64; do
    IGP_AB_AHEAD=$k step a${k}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/a${k}_$i.json
  done
done
