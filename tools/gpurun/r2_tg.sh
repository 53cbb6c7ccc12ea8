#!/bin/bash
# cfg3 tree-group count A/B (IGP_TREE_GROUPS; default picks 4 at 8192 rows), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2tg
mkdir -p $O
for pass in 1 2; do
  for g in 0 2 8 12; do
    IGP_TREE_GROUPS=$g timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_g${g}_$pass.json > $O/cfg3_g${g}_$pass.log 2>&1 || exit 1
  done
done
