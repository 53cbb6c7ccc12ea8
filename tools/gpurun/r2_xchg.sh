#!/bin/bash
# the DP serving path at world 1 (RCCL single-rank exchange) at HEAD, and cfg5 / cfg4 defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/xchg
mkdir -p $O
IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/xchg.json > $O/xchg.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3.json > $O/cfg3.log 2>&1 || exit 2
