#!/bin/bash
# exchange path with direct launch: DP GPU tests; world-1 exchange bench direct vs graphs;
# async issue x direct launch on cfg3 / cfg2 / heuristic (two passes, same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2direct3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py tests/test_engine_gpu.py tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_dp.log 2>&1 || exit 1
for x in 1 0 1 0; do
  IGP_DIRECT_LAUNCH=$x timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 --json-out $O/cfg4_d$x.json > $O/cfg4_d$x.log 2>&1 || exit 5
done
for x in 1 0 1 0; do
  IGP_DIRECT_LAUNCH=$x IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/xchg_d$x.json > $O/xchg_d$x.log 2>&1 || exit 2
done
for pass in 1 2; do
  for x in 0 1; do
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_a${x}_p$pass.json > $O/cfg3_a${x}_p$pass.log 2>&1 || exit 3
    IGP_ASYNC_SUBMIT=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_a${x}_p$pass.json > $O/cfg2_a${x}_p$pass.log 2>&1 || exit 4
  done
done
