#!/bin/bash
# Round 5: exchange path with recorded state / model stages: dp tests, N = 1 A/B, HIP API trace.
set -o pipefail
O=gpurun_out/r5al
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
export IGP_BENCH_SPMD=1
for i in 1 2 3; do
  for m in d2h a2a; do
    IGP_XCHG_RESULTS=$m step x_${m}_$i 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/x_${m}_$i.json
  done
done
cd /tmp
IGP_XCHG_RESULTS=d2h step prof 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof -o run -- python $R/bench.py --steps 4 --warmup 2 --json-out $R/$O/prof.json
