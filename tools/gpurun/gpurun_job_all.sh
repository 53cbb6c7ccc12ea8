#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/res
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
for c in cfg3 cfg2 cfg4 cfg5 heuristic; do
  timeout -k 10 300 python bench.py --config $c --json-out gpurun_out/res/bench_${c}_1gpu.json > gpurun_out/res/bench_$c.log 2>&1 || exit 3
done
