#!/bin/bash
# split state stage (model waits K1 only): parity tests, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2split
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_split.log 2>&1 || exit 1
for pass in 1 2 3; do
  for x in 0 1; do
    IGP_SPLIT_STATE=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_s${x}_$pass.json > $O/cfg3_s${x}_$pass.log 2>&1 || exit 2
  done
done
for x in 0 1; do
  IGP_SPLIT_STATE=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_s${x}.json > $O/cfg2_s${x}.log 2>&1 || exit 3
done
