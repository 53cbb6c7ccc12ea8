#!/bin/bash
# Round 4 seventh pass: cfg4 layer-kernel phase trace + design comparison; the account-RPC
# open-loop curves re-run at the fp32 defaults (PredictLTV, GetPlayerSegment, CheckBonusAbuse).
set -o pipefail
O=gpurun_out/r4g
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -3 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step acct_tests 300 python -u -m pytest tests/test_acct_gpu.py tests/test_mlp_fused_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider
export OUT=$R/$O/mlp_trace.json
step trace 200 python tools/mlp_layerwise_bench.py 8192 --trace
export OUT=$R/$O/mlp_layerwise.json
step layerwise 300 python tools/mlp_layerwise_bench.py 8192,16384
cd /tmp
export OUT=/tmp/lw.json
step prof_cfg4 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_cfg4 -o lw -- python $R/tools/mlp_layerwise_bench.py 8192
cd $R
for rpc in ltv segment abuse; do
  step curve_$rpc 400 python -u tools/bench_e2e.py --scope grpc --rpc $rpc --open-loop --rates 50000,100000,150000,200000 \
    --seconds 4 --clients 8 --json-out $R/$O/${rpc}_curve.json
done
