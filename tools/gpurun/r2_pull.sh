#!/bin/bash
# kernel pull-copy for the stage copies (IGP_PULL_COPY): correctness, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2pull
mkdir -p $O
IGP_PULL_COPY=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_pull.log 2>&1 || exit 1
for pass in 1 2; do
  for x in 0 1; do
    IGP_PULL_COPY=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_p${x}_$pass.json > $O/cfg3_p${x}_$pass.log 2>&1 || exit 2
    IGP_PULL_COPY=$x IGP_LTV_DIRECT=1 timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 --json-out $O/cfg4d_p${x}_$pass.json > $O/cfg4d_p${x}_$pass.log 2>&1 || exit 3
    IGP_PULL_COPY=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_p${x}_$pass.json > $O/cfg2_p${x}_$pass.log 2>&1 || exit 4
  done
  timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 --json-out $O/cfg4g_$pass.json > $O/cfg4g_$pass.log 2>&1 || exit 5
done
