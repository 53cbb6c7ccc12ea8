#!/bin/bash
# Round 6: kernel statistics of engine_only and serving after the tree traversal rework.
set -o pipefail
O=gpurun_out/r6m
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
step prof_eng 400 rocprofv3 --kernel-trace --stats -d $R/$O/eng -o eng -- python bench.py --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/prof_eng.json
step prof_srv 400 rocprofv3 --kernel-trace --stats -d $R/$O/srv -o srv -- python bench.py --steps 20 --warmup 5 --json-out $R/$O/prof_srv.json
