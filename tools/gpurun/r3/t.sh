#!/bin/bash
# round 3, pass t: chain-kernel k-step rotation A/B (standalone launches), the driver's exact bench
# command with the serving-step definition (one request per ingress thread per step), mlp tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3t
mkdir -p $O
for kr in 0 1 0 1; do
  IGP_MLP_KROT=$kr OUT=$O/mlp_krot$kr.json timeout -k 10 200 python tools/mlp_bench.py 8192,16384 > $O/mlp_krot$kr.log 2>&1 || exit 3
  echo "krot=$kr" >> $O/status.txt
  grep -v amdgpu.ids $O/mlp_krot$kr.log | grep -v '"pair"' | cut -c1-100 >> $O/status.txt
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/driver_cmd_$i.json > $O/driver_cmd_$i.log 2>&1 || exit 4
  echo "driver cmd $(python -c "import json;d=json.load(open('$O/driver_cmd_$i.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2),'ms/step',round(d['ms_per_step'],2))")" >> $O/status.txt
done
timeout -k 10 300 python -u -m pytest tests/test_mlp_fused_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
echo "tests rc=$?" >> $O/status.txt
