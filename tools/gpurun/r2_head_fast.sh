#!/bin/bash
# specialised f32 MLP head: GPU suite, same-box A/B against the generic kernel (IGP_HEAD_GENERIC),
# per-kernel times and the head's phase trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for g in 0 1; do
    IGP_HEAD_GENERIC=$g timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_g${g}_$i.json > $O/cfg3_g${g}_$i.log 2>&1 || exit 2
  done
done
timeout -k 10 200 python tools/kbench.py --config cfg3 --rounds 40 --only mlp_head,tree_ensemble --out $O/kbench.json > $O/kbench.log 2>&1 || exit 3
IGP_HEAD_GENERIC=1 timeout -k 10 200 python tools/kbench.py --config cfg3 --rounds 40 --only mlp_head --out $O/kbench_generic.json > $O/kbench_generic.log 2>&1 || exit 4
