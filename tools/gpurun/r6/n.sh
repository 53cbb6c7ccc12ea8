#!/bin/bash
# Round 6: account-router benches (cfg5 / cfg4) over the device pipeline depth, stepper woken only when needed.
set -o pipefail
O=gpurun_out/r6n
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
for d in 2 3 4; do
  step cfg5_d$d 300 python bench.py --config cfg5 --steps 5 --warmup 1 --depth $d --json-out $R/$O/cfg5_d$d.json
done
for d in 2 3; do
  step cfg4_d$d 300 python bench.py --config cfg4 --steps 5 --warmup 1 --depth $d --json-out $R/$O/cfg4_d$d.json
done
step cfg5_d3_b 300 python bench.py --config cfg5 --steps 5 --warmup 1 --depth 3 --json-out $R/$O/cfg5_d3_b.json
step cfg5_d3_t4 300 python bench.py --config cfg5 --steps 5 --warmup 1 --depth 3 --drive-threads 4 --json-out $R/$O/cfg5_d3_t4.json
step cfg4_d3_t4 300 python bench.py --config cfg4 --steps 5 --warmup 1 --depth 3 --drive-threads 4 --json-out $R/$O/cfg4_d3_t4.json
