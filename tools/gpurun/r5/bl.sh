#!/bin/bash
# Round 5: cfg4 / cfg5 engine_only at HEAD, cfg4 kernel statistics.
set -o pipefail
O=gpurun_out/r5bl
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
  step cfg4_eng_$i 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_eng_$i.json
  step cfg5_eng_$i 300 python bench.py --config cfg5 --scope engine_only --steps 20 --warmup 3 --json-out $R/$O/cfg5_eng_$i.json
done
cd /tmp
step prof4 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof4 -o run -- python $R/bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/prof4.json
