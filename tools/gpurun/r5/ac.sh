#!/bin/bash
# Round 5: exchange path at N = 1 - header folded into the clear kernel, results scattered
# straight into the node-shared pinned region (d2h mode); dp GPU tests, then a2a vs d2h serving.
set -o pipefail
O=gpurun_out/r5ac
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
step dp_tests 400 python -u -m pytest tests/test_dp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  for m in a2a d2h; do
    IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=$m step spmd_${m}_$i 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_${m}_$i.json
  done
done
(cd /tmp && IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- \
  python $R/bench.py --steps 3 --warmup 2 --rounds 8 > $R/$O/prof.log 2>&1)
echo "prof rc=$?" >> $R/$O/status.txt
