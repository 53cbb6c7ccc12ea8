#!/bin/bash
# Round 6: serving abuse device with 32-row split-GRU tiles for the 4096-row bucket - account
# GPU tests, cfg5 through the router (1 / 4 drive threads), mixed traffic.
set -o pipefail
O=gpurun_out/r6t
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
step tests 400 python -u -m pytest tests/test_acct_gpu.py tests/test_gru_gpu.py -x -v --timeout 120 --timeout-method thread
for t in 1 4; do
  for i in 1 2; do
    step cfg5_t${t}_$i 300 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads $t --json-out $R/$O/cfg5_t${t}_$i.json
  done
done
step cfg5_t1_3 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_t1_3.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
