#!/bin/bash
# Round 5: the exchange (multi-GPU) serving path at N = 1, the account-router benches with 4
# submit threads, cfg5 engine_only fp32 / bf16.
set -o pipefail
O=gpurun_out/r5aa
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
IGP_BENCH_SPMD=1 step spmd 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd.json
step cfg5 400 python bench.py --config cfg5 --steps 20 --warmup 3 --json-out $R/$O/cfg5.json
step cfg4 400 python bench.py --config cfg4 --steps 20 --warmup 3 --json-out $R/$O/cfg4.json
step cfg5_eng 400 python bench.py --config cfg5 --scope engine_only --steps 40 --warmup 10 --json-out $R/$O/cfg5_eng.json
step cfg5_eng_bf16 400 python bench.py --config cfg5 --scope engine_only --numerics bf16 --steps 40 --warmup 10 --json-out $R/$O/cfg5_eng_bf16.json
step cfg4_eng 400 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_eng.json
