#!/bin/bash
# round 3, pass p: chain-kernel weight prefetch depth sweep (standalone launches), GRU placement trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3p
mkdir -p $O
for cfg in "5 4" "8 8" "10 12" "0 0"; do
  set -- $cfg
  IGP_MC_PF=$1 IGP_MP_PF=$2 OUT=$O/mlp_pf$1_$2.json timeout -k 10 200 python tools/mlp_bench.py 8192,16384 > $O/mlp_pf$1_$2.log 2>&1 || exit 3
  echo "mc_pf=$1 mp_pf=$2" >> $O/status.txt
  grep -v amdgpu.ids $O/mlp_pf$1_$2.log | cut -c1-110 >> $O/status.txt
done
timeout -k 10 120 python tools/gru_ws_trace.py 4096 3 > $O/gru_trace_ws3.txt 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest tests/test_mlp_fused_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
echo "tests rc=$?" >> $O/status.txt
