#!/bin/bash
# round 3, pass zg: serving pipeline slots 3 vs 5, interleaved, 200 steps each (host stages and
# device latency recorded per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3zg
mkdir -p $O
for i in 1 2 3; do
  for d in 3 5; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 5 --depth $d --json-out $O/serve_d${d}_$i.json > $O/serve_d${d}_$i.log 2>&1 || exit 6
    echo "serve depth $d $(python -c "import json;d=json.load(open('$O/serve_d${d}_$i.json'));h=d['host_stages_rank0'];print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2),'dev_us',h['device_us_per_step'],'resolve',h['resolve_ns_per_row'],'copy',h['copy_ns_per_row'])")" >> $O/status.txt
  done
done
