#!/bin/bash
# GRU cluster kernel with the two-half hand-off pipeline (ws=2 / IGP_GRU_SPLIT): parity tests,
# then a same-box cfg5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/grusplit
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
for i in 1 2; do
  for p in 1 0; do
    IGP_GRU_SPLIT=$p timeout -k 10 200 python bench.py --config cfg5 --steps 300 --warmup 30 --json-out $O/cfg5_split${p}_$i.json > $O/cfg5_split${p}_$i.log 2>&1 || exit 2
  done
done
