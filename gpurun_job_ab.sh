#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
for v in 1 0 1 0 1 0; do
  IGP_HOST_RESULTS=$v timeout -k 10 200 python bench.py --steps 400 --warmup 50 > gpurun_out/ab/b_$v.log 2>&1 || exit 5
  echo "hostres=$v $(tail -1 gpurun_out/ab/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p99_latency_ms"], d["host_us_per_batch"]["wait_us"])')" >> gpurun_out/ab/summary.txt
done
