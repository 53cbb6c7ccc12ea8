#!/bin/bash
# f32 head with K padded to 32: head / engine GPU tests, head phase trace, cfg3 bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/kpad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
timeout -k 10 200 python tools/kbench.py --config cfg3 --rounds 40 --only mlp_head,tree_ensemble --out $O/kbench.json > $O/kbench.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_$i.json > $O/cfg3_$i.log 2>&1 || exit 3
done
