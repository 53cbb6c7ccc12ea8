#!/bin/bash
# cfg3 CU-split A/B: state+copy side size (lo:N, CU index order) and interleaved (mod:1/2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2cu
mkdir -p $O
for pass in 1 2; do
  for sp in half lo:96 lo:112 lo:144 mod:1/2 none; do
    n=$(echo $sp | tr ':/' '__')
    IGP_CU_SPLIT=$sp timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_${n}_$pass.json > $O/cfg3_${n}_$pass.log 2>&1 || exit 1
  done
done
