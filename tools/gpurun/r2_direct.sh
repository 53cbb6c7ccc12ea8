#!/bin/bash
# direct-launch driver mode: parity tests, then same-box A/B vs graph replay (cfg3, cfg2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2direct
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_gpu.log 2>&1 || exit 1
for pass in 1 2; do
  for x in 0 1; do
    IGP_DIRECT_LAUNCH=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_d${x}_p$pass.json > $O/cfg3_d${x}_p$pass.log 2>&1 || exit 2
    IGP_DIRECT_LAUNCH=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_d${x}_p$pass.json > $O/cfg2_d${x}_p$pass.log 2>&1 || exit 3
  done
done
