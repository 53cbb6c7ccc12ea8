#!/bin/bash
# Round 6: K1 amount-ring loads as 16-byte pairs (B) vs one 8-byte load per entry (A), same box,
# interleaved serving / engine_only runs; cfg5 account-router bench over the in-flight window;
# cfg4 per-thread CPU with 2 / 4 finishers.
set -o pipefail
O=gpurun_out/r6r
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
SO=$R/igaming_platform_amd/_hipk.cpython-310-x86_64-linux-gnu.so
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2 3; do
  for v in A B; do
    cp $R/ab/_hipk_$v.so $SO
    step srv_${v}$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_${v}$i.json
    step eng_${v}$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_${v}$i.json
  done
done
cp $R/ab/_hipk_B.so $SO
for w in 16384 32768 49152; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg5_w${w}_threads.json step cfg5_w$w 300 python bench.py --config cfg5 --steps 5 --warmup 1 --inflight $w --json-out $R/$O/cfg5_w$w.json
done
for f in 2 4; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg4_f${f}_threads.json step cfg4_f$f 300 python bench.py --config cfg4 --steps 5 --warmup 1 --drive-threads 4 --finishers $f --json-out $R/$O/cfg4_f$f.json
done
