#!/bin/bash
# Round 4 fourth pass: ai.onnx.ml linear pipelines + DAG joins on the device, the world-1
# exchange ordering test, account-RPC GPU tests, tree kernels (PROBIT edge fix).
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a crash / abort / time limit
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt; tail -3 $O/$name.log >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step tests 900 python -u -m pytest tests/test_onnx_ml_gpu.py tests/test_dp_gpu.py tests/test_acct_gpu.py \
  tests/test_kernels_gpu.py tests/test_mlp_fused_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider
# BASELINE config 1: ScoreTransaction through the native HTTP/2 server on the C++ CPU backend
# (32-feature logistic, no GPU), open loop
step cfg1_curve 600 python -u tools/bench_e2e.py --scope grpc --rpc tx --open-loop --backend cpu --model cfg1 \
  --rates 5000,20000,50000,100000,150000,200000 --seconds 4 --clients 8 --json-out $O/cfg1_curve.json
