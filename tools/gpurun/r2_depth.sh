#!/bin/bash
# cfg3 pipeline depth A/B (batches in flight = pipeline slots), same box, two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2depth
mkdir -p $O
for pass in 1 2; do
  for d in 3 4 5 6; do
    timeout -k 10 200 python bench.py --depth $d --steps 400 --warmup 40 --json-out $O/bench_d${d}_p$pass.json > $O/bench_d${d}_p$pass.log 2>&1 || exit 1
  done
done
