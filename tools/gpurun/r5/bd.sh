#!/bin/bash
# Round 5 (experiment): one pipeline stream at high priority (state / model / copy) vs none.
set -o pipefail
O=gpurun_out/r5bd
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
  for p in none state model copy; do
    IGP_AB_PRIO=$p step eng_${p}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_${p}_$i.json
  done
done
for i in 1 2; do
  for p in none state model; do
    IGP_AB_PRIO=$p step srv_${p}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_${p}_$i.json
  done
done
