#!/bin/bash
# Round 5 (end): kernel statistics of the driver's serving bench and of engine_only at HEAD.
set -o pipefail
O=gpurun_out/r5bi
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
cd /tmp
step prof_srv 300 rocprofv3 --kernel-trace --stats -d $R/$O/srv -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/srv.json
step prof_eng 300 rocprofv3 --kernel-trace --stats -d $R/$O/eng -o run -- python $R/bench.py --scope engine_only --steps 300 --warmup 20 --json-out $R/$O/eng.json
