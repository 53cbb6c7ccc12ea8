#!/bin/bash
# Round 5: split GRU clusters - per-step phase trace and kernel times vs the batch-parallel kernel,
# then the GRU GPU tests.
set -o pipefail
O=gpurun_out/r5x
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
step trace 240 python tools/gru_wsx_trace.py --rows 32
step gru_tests 400 python -u -m pytest tests/test_gru_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "split"
