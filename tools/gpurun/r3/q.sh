#!/bin/bash
# round 3, pass q: device-encoded FeatureVector bodies (K1 write_fenc) - engine / kernel GPU tests,
# serving bench A/B (IGP_FEAT_ENC 1 vs 0); chain-kernel prefetch depth sweep; GRU placement trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_dp_gpu.py tests/test_mlp_fused_gpu.py -m gpu -v -x --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
for fe in 1 0 1 0; do
  IGP_FEAT_ENC=$fe timeout -k 10 300 python bench.py --steps 400 --warmup 40 --json-out $O/serving_enc$fe.json > $O/serving_enc$fe.log 2>&1 || exit 3
  echo "serving enc=$fe $(python -c "import json;d=json.load(open('$O/serving_enc$fe.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2), d['host_stages_rank0'])")" >> $O/status.txt
done
for cfg in "5 4" "8 8" "0 0"; do
  set -- $cfg
  IGP_MC_PF=$1 IGP_MP_PF=$2 OUT=$O/mlp_pf$1_$2.json timeout -k 10 200 python tools/mlp_bench.py 8192,16384 > $O/mlp_pf$1_$2.log 2>&1 || exit 4
  echo "mc_pf=$1 mp_pf=$2" >> $O/status.txt
  grep -v amdgpu.ids $O/mlp_pf$1_$2.log | cut -c1-110 >> $O/status.txt
done
timeout -k 10 120 python tools/gru_ws_trace.py 4096 3 > $O/gru_trace_ws3.txt 2>&1 || exit 5
