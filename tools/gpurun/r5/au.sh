#!/bin/bash
# Round 5: engine_only cfg3 kernel + HIP API trace (where the 59 us per 8192-row batch goes).
set -o pipefail
O=gpurun_out/r5au
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
step prof 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof -o run -- python $R/bench.py --scope engine_only --steps 300 --warmup 20 --json-out $R/$O/prof.json
cd $R
for i in 1 2; do
  for cs in none half lo:96 lo:160; do
    n=$(echo $cs | tr ':' '_')
    IGP_CU_SPLIT=$cs step eng_${n}_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_${n}_$i.json
  done
done
for i in 1 2; do
  for cs in none half; do
    IGP_CU_SPLIT=$cs step srv_${cs}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_${cs}_$i.json
  done
done
