#!/bin/bash
# pipeline depth 3 vs 4 at HEAD (bound stage events, fused cfg2 ensemble), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/depth2
mkdir -p $O
for i in 1 2; do
  for d in 3 4; do
    timeout -k 10 200 python bench.py --depth $d --steps 2000 --warmup 100 --json-out $O/cfg3_d${d}_$i.json > $O/cfg3_d${d}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --config cfg2 --depth $d --steps 2000 --warmup 100 --json-out $O/cfg2_d${d}_$i.json > $O/cfg2_d${d}_$i.log 2>&1 || exit 2
  done
done
