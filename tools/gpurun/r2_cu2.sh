#!/bin/bash
# cfg3 CU split half vs none (direct launch), 5 interleaved passes, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2cu3
mkdir -p $O
for pass in 1 2 3; do
  for sp in half none; do
    IGP_CU_SPLIT=$sp timeout -k 10 200 python bench.py --steps 3000 --warmup 100 --json-out $O/cfg3_${sp}_$pass.json > $O/cfg3_${sp}_$pass.log 2>&1 || exit 1
  done
done
