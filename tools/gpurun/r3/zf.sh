#!/bin/bash
# round 3, pass zf: pipeline depth (slots / streams) A/B for cfg5 fp32 and cfg4 fp32: 3 vs 4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3zf
mkdir -p $O
for i in 1 2; do
  for d in 3 4; do
    timeout -k 10 250 python bench.py --config cfg5 --depth $d --steps 60 --warmup 10 --json-out $O/cfg5_d${d}_$i.json > $O/cfg5_d${d}_$i.log 2>&1 || exit 4
    echo "cfg5 fp32 depth $d $(python -c "import json;d=json.load(open('$O/cfg5_d${d}_$i.json'));print(round(d['value']/1e6,3),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', round(d.get('p99_latency_ms'),3))")" >> $O/status.txt
    timeout -k 10 200 python bench.py --config cfg4 --depth $d --steps 300 --warmup 20 --json-out $O/cfg4_d${d}_$i.json > $O/cfg4_d${d}_$i.log 2>&1 || exit 5
    echo "cfg4 fp32 depth $d $(python -c "import json;d=json.load(open('$O/cfg4_d${d}_$i.json'));print(round(d['value']/1e6,2),'M/s', round(d['ms_per_step']*1e3,1),'us/step p99', round(d.get('p99_latency_ms'),3))")" >> $O/status.txt
  done
done
