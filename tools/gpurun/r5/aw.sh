#!/bin/bash
# Round 5: serving A/B, per-thread reused request-row buffer vs a fresh vector per request.
set -o pipefail
O=gpurun_out/r5aw
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
  step reuse_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/reuse_$i.json
  IGP_AB_FRESH_ROWS=1 step fresh_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/fresh_$i.json
done
IGP_BENCH_SAMPLE=1 IGP_BENCH_THREADS_OUT=$R/$O/hot_plain.json step hot_plain 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/hot_plain_b.json
