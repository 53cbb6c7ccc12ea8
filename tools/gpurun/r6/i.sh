#!/bin/bash
# Round 6: split GRU cluster stalls in the serving abuse device - counter-reset memset A/B;
# cfg5 serving with the clusters off (default); mixed traffic; tree phase trace.
set -o pipefail
O=gpurun_out/r6i
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
# pytest failures (rc 1) are results here; anything else ends the job
tstep() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
}
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
tstep t_reset 300 $T tests/test_acct_gpu.py -k cluster_kernel_option
tstep t_noreset 300 env IGP_GRU_NO_RESET=1 $T tests/test_acct_gpu.py -k cluster_kernel_option
step cfg5_t1 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1.json
step cfg5_t1_on_noreset 300 env IGP_GRU_NO_RESET=1 python tools/nowsx.py --serving-on bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1_on_noreset.json
step cfg5_t8 300 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg5_t8.json
step tree_bench 200 python tools/tree_bench.py
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
