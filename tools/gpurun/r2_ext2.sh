#!/bin/bash
# stage-end events: bound-to-kernel (IGP_EXT_EVENTS) x device-scope fences (IGP_EVENT_DEVSCOPE),
# same-box A/B of cfg3 (twice) and cfg2; then the per-kernel times and the head's phase trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ext2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "direct_launch or pipelined" > $O/t.log 2>&1 || exit 1
for i in 1 2; do
  for v in "1 1" "0 1" "1 0" "0 0"; do
    set -- $v
    IGP_EXT_EVENTS=$1 IGP_EVENT_DEVSCOPE=$2 timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_x$1_d$2_$i.json > $O/cfg3_x$1_d$2_$i.log 2>&1 || exit 2
  done
done
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  IGP_EXT_EVENTS=$1 IGP_EVENT_DEVSCOPE=$2 timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --json-out $O/cfg2_x$1_d$2.json > $O/cfg2_x$1_d$2.log 2>&1 || exit 3
done
timeout -k 10 200 python tools/kbench.py --config cfg3 --rounds 40 --only mlp_head,tree_ensemble,feature_assemble+single_update,dedup_insert --out $O/kbench.json > $O/kbench.log 2>&1 || exit 4
