#!/bin/bash
# Round 5: account-router bench (cfg5 / cfg4) with the single-thread submit+poll drive loop.
set -o pipefail
O=gpurun_out/r5bb
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
  step cfg5_$i 400 python bench.py --config cfg5 --steps 20 --warmup 5 --json-out $R/$O/cfg5_$i.json
  step cfg4_$i 400 python bench.py --config cfg4 --steps 20 --warmup 5 --json-out $R/$O/cfg4_$i.json
done
step cfg5_t2 400 python bench.py --config cfg5 --steps 20 --warmup 5 --drive-threads 2 --json-out $R/$O/cfg5_t2.json
