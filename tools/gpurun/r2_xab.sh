#!/bin/bash
# world-1 exchange A/Bs: direct state stage (IGP_XCHG_STATE_DIRECT) and CU split, 2000 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2xab
mkdir -p $O
export IGP_FORCE_EXCHANGE=1
IGP_XCHG_STATE_DIRECT=1 timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
for pass in 1 2; do
  for v in "0 auto" "1 auto" "0 none" "1 none"; do
    set -- $v
    IGP_XCHG_STATE_DIRECT=$1 IGP_CU_SPLIT=$2 timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/x_sd$1_$2_$pass.json > $O/x_sd$1_$2_$pass.log 2>&1 || exit 2
  done
done
