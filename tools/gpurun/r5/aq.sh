#!/bin/bash
# Round 5: exchange scorer at serve_depth (was pinned to 3): dp tests, N = 1 A/B vs plain.
set -o pipefail
O=gpurun_out/r5aq
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
  for m in d2h a2a; do
    IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=$m step x_${m}_$i 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/x_${m}_$i.json
  done
  IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h step x_d2h_d6_$i 300 python bench.py --steps 40 --warmup 5 --depth 6 --json-out $R/$O/x_d2h_d6_$i.json
  step plain_$i 300 python bench.py --steps 40 --warmup 5 --json-out $R/$O/plain_$i.json
done
