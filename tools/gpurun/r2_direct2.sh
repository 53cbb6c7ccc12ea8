#!/bin/bash
# direct launch (default now) x async issue A/B: cfg2 / cfg3, two passes, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2direct2
mkdir -p $O
for pass in 1 2; do
  for x in 0 1; do
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_a${x}_p$pass.json > $O/cfg3_a${x}_p$pass.log 2>&1 || exit 2
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_a${x}_p$pass.json > $O/cfg2_a${x}_p$pass.log 2>&1 || exit 3
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --config heuristic --steps 400 --warmup 40 --json-out $O/heur_a${x}_p$pass.json > $O/heur_a${x}_p$pass.log 2>&1 || exit 4
  done
done
