#!/bin/bash
# Round 6: baseline at HEAD - driver command, SPMD world-1 path, cfg4 / cfg5 engine depth 3 vs 4, cfg2.
set -o pipefail
O=gpurun_out/r6a
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
step bench 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
IGP_BENCH_SPMD=1 step spmd 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd.json
for d in 3 4; do
  step cfg4_d$d 300 python bench.py --config cfg4 --scope engine_only --depth $d --steps 200 --warmup 20 --json-out $R/$O/cfg4_d$d.json
  step cfg5_d$d 300 python bench.py --config cfg5 --scope engine_only --depth $d --steps 20 --warmup 3 --json-out $R/$O/cfg5_d$d.json
done
step cfg2 300 python bench.py --config cfg2 --steps 20 --warmup 5 --json-out $R/$O/cfg2.json
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
