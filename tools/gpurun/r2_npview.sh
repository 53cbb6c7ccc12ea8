#!/bin/bash
# result readback through precomputed numpy views: engine GPU tests + default bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/npview
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_$i.json > $O/cfg3_$i.log 2>&1 || exit 2
done
