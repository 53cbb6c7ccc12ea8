#!/bin/bash
# Round 6: GPU suite + smoke after the ADVICE fixes (clock retract, cluster counter reset, wsx / multi-stream).
set -o pipefail
O=gpurun_out/r6b
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
