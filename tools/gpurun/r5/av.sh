#!/bin/bash
# Round 5: serving host profile (per-thread CPU + hottest functions) and serving runs after the
# link-queue change.
set -o pipefail
O=gpurun_out/r5av
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
IGP_BENCH_SAMPLE=1 IGP_BENCH_THREADS_OUT=$R/$O/hot_plain.json step hot_plain 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/hot_plain_b.json
IGP_BENCH_SPMD=1 IGP_BENCH_SAMPLE=1 IGP_BENCH_THREADS_OUT=$R/$O/hot_spmd.json step hot_spmd 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/hot_spmd_b.json
for i in 1 2 3; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
done
