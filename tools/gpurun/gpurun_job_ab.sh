#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
cd $GRAFT_REPO_ROOT
for v in 3 4 5 3 4 5; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 50 --depth $v > gpurun_out/ab/b_x.log 2>&1 || exit 5
  echo "depth=$v $(tail -1 gpurun_out/ab/b_x.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p99_latency_ms"], d["host_us_per_batch"]["wait_us"])')" >> gpurun_out/ab/summary.txt
done
