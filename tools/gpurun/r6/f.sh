#!/bin/bash
# Round 6: account-RPC bench diagnostics (device time per step, cluster fallbacks) at HEAD;
# mixed traffic with unary-first steps, high-priority abuse streams, abuse step cap.
set -o pipefail
O=gpurun_out/r6f
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
step cfg5_srv_t1 400 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5_srv_t1.json
step cfg5_srv_t8 400 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg5_srv_t8.json
step cfg4_srv_t8 400 python bench.py --config cfg4 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg4_srv_t8.json
step mixed_closed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_closed.json
step mixed_closed_cap256 400 python tools/bench_mixed.py --seconds 5 --abuse-max-batch 256 --json-out $R/$O/mixed_closed_cap256.json
step mixed_open 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --json-out $R/$O/mixed_open.json
step mixed_open_cap256 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --abuse-max-batch 256 --json-out $R/$O/mixed_open_cap256.json
step mixed_open_noprio 400 python tools/bench_mixed.py --seconds 5 --batch-rate 6000 --abuse-priority 0 --json-out $R/$O/mixed_open_noprio.json
