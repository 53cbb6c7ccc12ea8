#!/bin/bash
# Round 6: cfg5 serving regression - kernel trace, same-box A/B without the split GRU clusters;
# mixed traffic with the abuse time breakdown (normal priority).
set -o pipefail
O=gpurun_out/r6g
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
step cfg5_t1 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1.json
step cfg5_t1_nowsx 300 python tools/nowsx.py bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1_nowsx.json
step cfg5_prof 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o cfg5 -- python bench.py --config cfg5 --steps 3 --warmup 1 --json-out $R/$O/cfg5_prof.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
