#!/bin/bash
# stage-end events bound to the stages' last kernels (IGP_EXT_EVENTS): parity tests, then a
# same-box A/B of the default cfg3 bench (alternating, 2000 steps each)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ext
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "direct_launch or pipelined" > $O/t.log 2>&1 || exit 1
for i in 1 2; do
  for x in 1 0; do
    IGP_EXT_EVENTS=$x timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_ext${x}_$i.json > $O/cfg3_ext${x}_$i.log 2>&1 || exit 2
  done
done
for x in 1 0; do
  IGP_EXT_EVENTS=$x timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --json-out $O/cfg2_ext${x}.json > $O/cfg2_ext${x}.log 2>&1 || exit 3
done
