#!/bin/bash
# diagnostic: cfg3 throughput vs micro-batch size (host / launch overhead per batch vs GPU work)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2bdiag
mkdir -p $O
for b in 4096 8192 16384 8192; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 --json-out $O/bench_b$b.json > $O/bench_b$b.log 2>&1 || exit 1
done
