#!/bin/bash
# Round 5: exchange serving path at N = 1: captured graphs vs direct launch (recorded op lists),
# a2a vs node-shared results; dp GPU tests first (incl. direct + d2h).
set -o pipefail
O=gpurun_out/r5af
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
IGP_XCHG_DIRECT=1 IGP_XCHG_RESULTS=d2h step dp_tests_direct_d2h 400 python -u -m pytest tests/test_dp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "world1_matches"
for i in 1 2; do
  for dm in 0 1; do
    for m in a2a d2h; do
      IGP_XCHG_DIRECT=$dm IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=$m step spmd_x${dm}_${m}_$i 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_x${dm}_${m}_$i.json
    done
  done
done
IGP_BENCH_THREADS_OUT=$R/$O/threads_plain.json step thr_plain 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/thr_plain.json
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h IGP_BENCH_THREADS_OUT=$R/$O/threads_spmd.json step thr_spmd 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/thr_spmd.json
