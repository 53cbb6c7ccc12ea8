#!/bin/bash
# async driver issue A/B (IGP_ASYNC_SUBMIT), cfg3 + cfg2, two passes, same box; engine GPU tests
# with async issue on
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2async
mkdir -p $O
IGP_ASYNC_SUBMIT=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine_async.log 2>&1 || exit 1
for pass in 1 2; do
  for x in 0 1; do
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_a${x}_p$pass.json > $O/cfg3_a${x}_p$pass.log 2>&1 || exit 2
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_a${x}_p$pass.json > $O/cfg2_a${x}_p$pass.log 2>&1 || exit 3
  done
done
