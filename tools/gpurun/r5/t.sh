#!/bin/bash
# Round 5: unary ScoreTransaction / PredictLTV / CheckBonusAbuse over the native HTTP/2 server on
# the GPU backend - open-loop rates, per-thread-group CPU cost per call (tools/host_profile.py).
set -o pipefail
O=gpurun_out/r5t
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
echo "nproc $(nproc) affinity $(python -c 'import os; print(len(os.sched_getaffinity(0)))')" >> $R/$O/status.txt
for rate in 100000 200000 300000 400000 500000 600000; do
  step tx_w8_$rate 240 python tools/host_profile.py --backend gpu --model cfg3 --rpc tx --rate $rate --seconds 3 --clients 8 --workers 8 --json-out $R/$O/tx_w8_$rate.json
done
step tx_w12_500000 240 python tools/host_profile.py --backend gpu --model cfg3 --rpc tx --rate 500000 --seconds 3 --clients 8 --workers 12 --json-out $R/$O/tx_w12_500000.json
step tx_sample 240 python tools/host_profile.py --backend gpu --model cfg3 --rpc tx --rate 300000 --seconds 3 --clients 8 --workers 8 --sample --json-out $R/$O/tx_sample.json
for rpc in abuse ltv; do
  for rate in 100000 200000 300000; do
    step ${rpc}_$rate 300 python tools/host_profile.py --backend gpu --rpc $rpc --rate $rate --seconds 3 --clients 8 --workers 8 --json-out $R/$O/${rpc}_$rate.json
  done
done
