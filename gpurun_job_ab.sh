#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k1_tests.log 2>&1 || exit 3
for v in auto none auto none; do
  export IGP_CU_SPLIT=$v
  timeout -k 10 200 python bench.py --config cfg2 --steps 800 --warmup 50 > gpurun_out/ab/b_x.log 2>&1 || exit 5
  echo "cfg2 split=$v $(tail -1 gpurun_out/ab/b_x.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p99_latency_ms"])')" >> gpurun_out/ab/summary.txt
done
