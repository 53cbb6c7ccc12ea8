#!/bin/bash
# round 3, pass s: serving A/B of the host wait policy (bounded 30-us spin + sleeps vs a ~5 ms spin
# like the old 4096-query loop), device-encoded features on; then the default bench x3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3s
mkdir -p $O
for sp in 30 5000 30 5000 30 5000 30 5000; do
  IGP_WAIT_SPIN_US=$sp timeout -k 10 300 python bench.py --steps 1500 --warmup 100 --json-out $O/serving_spin$sp.json > $O/serving_spin$sp.log 2>&1 || exit 3
  echo "serving spin_us=$sp $(python -c "import json;d=json.load(open('$O/serving_spin$sp.json'));print(round(d['value']/1e6,2),'M/s p50',round(d['p50_latency_ms'],2),'p99',round(d['p99_latency_ms'],2), d['host_stages_rank0'])")" >> $O/status.txt
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --json-out $O/default_$i.json > $O/default_$i.log 2>&1 || exit 4
  echo "default $(tail -c 420 $O/default_$i.json)" >> $O/status.txt
done
