#!/bin/bash
# round 3, pass r: serving A/B of device-encoded features over longer windows (2000 requests),
# GRU placement trace, cfg4 engine at the restored prefetch depth
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3r
mkdir -p $O
for fe in 1 0 1 0 1 0; do
  IGP_FEAT_ENC=$fe timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --json-out $O/serving_enc$fe.json > $O/serving_enc$fe.log 2>&1 || exit 3
  echo "serving enc=$fe $(python -c "import json;d=json.load(open('$O/serving_enc$fe.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2), d['host_stages_rank0'])")" >> $O/status.txt
done
timeout -k 10 120 python tools/gru_ws_trace.py 4096 3 > $O/gru_trace_ws3.txt 2>&1 || exit 4
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --numerics bf16 --steps 400 --warmup 40 --json-out $O/cfg4_bf16_$i.json > $O/cfg4_$i.log 2>&1 || exit 5
  echo "cfg4 bf16 $(python -c "import json;d=json.load(open('$O/cfg4_bf16_$i.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step')")" >> $O/status.txt
done
