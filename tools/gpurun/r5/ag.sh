#!/bin/bash
# Round 5: exchange serving path at N = 1 after removing the direct-launch mode: dp GPU tests,
# then a2a vs node-shared (d2h) results A/B, then per-thread host CPU of plain vs exchange path.
set -o pipefail
O=gpurun_out/r5ag
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
    IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=$m step spmd_${m}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_${m}_$i.json
  done
done
IGP_BENCH_THREADS_OUT=$R/$O/threads_plain.json step thr_plain 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/thr_plain.json
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h IGP_BENCH_THREADS_OUT=$R/$O/threads_spmd.json step thr_spmd 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/thr_spmd.json
