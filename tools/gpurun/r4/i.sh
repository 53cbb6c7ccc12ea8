#!/bin/bash
# Round 4: the SPMD world-1 ordering test after the account tests (the full suite's order).
set -o pipefail
O=gpurun_out/r4i
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -3 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step dp 600 python -u -m pytest tests/test_acct_gpu.py tests/test_dedup_gpu.py tests/test_dp_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider
