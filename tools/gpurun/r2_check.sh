#!/bin/bash
# quick check at HEAD: engine + DP GPU tests, default bench, world-1 exchange bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3.json > $O/cfg3.log 2>&1 || exit 2
IGP_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/xchg.json > $O/xchg.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3b.json > $O/cfg3b.log 2>&1 || exit 4
