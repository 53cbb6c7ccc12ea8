#!/bin/bash
# Round 6: cfg4 through the account router over the answer-writing threads (2 / 4 / 6
# finishers); cfg3 serving bench over the ingress threads (12 / 16 / 20 / 24).
set -o pipefail
O=gpurun_out/r6x
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
  for f in 2 4 6; do
    IGP_BENCH_THREADS_OUT=$R/$O/cfg4_f${f}_${i}_threads.json step cfg4_f${f}_$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --finishers $f --json-out $R/$O/cfg4_f${f}_$i.json
  done
done
for i in 1 2; do
  for t in 12 16 20 24; do
    step srv_t${t}_$i 300 python bench.py --steps 20 --warmup 5 --threads $t --json-out $R/$O/srv_t${t}_$i.json
  done
done
