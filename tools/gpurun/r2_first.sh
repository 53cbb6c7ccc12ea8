#!/bin/bash
# is the first bench process on a fresh box slower? the default bench 4x in a row
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2first
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --json-out $O/cfg3_run$i.json > $O/cfg3_run$i.log 2>&1 || exit 1
done
