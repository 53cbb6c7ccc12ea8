#!/bin/bash
# Round 5: exchange path at N = 1 with device-scope hop/state events; kernel + HIP API trace.
set -o pipefail
O=gpurun_out/r5ak
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
export IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h
for i in 1 2 3; do
  for cs in none half; do
    IGP_CU_SPLIT=$cs step cu_${cs}_$i 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/cu_${cs}_$i.json
  done
done
cd /tmp
IGP_CU_SPLIT=none step prof 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof -o run -- python $R/bench.py --steps 4 --warmup 2 --json-out $R/$O/prof.json
