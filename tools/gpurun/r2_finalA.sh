#!/bin/bash
# round-end validation A: the whole GPU suite, smoke(), and every BASELINE config on 1 GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for c in cfg3 cfg3 cfg2 cfg4 cfg5 heuristic; do
  timeout -k 10 300 python bench.py --config $c --steps 300 --warmup 30 --json-out $O/bench_$c.json >> $O/bench.log 2>&1 || exit 3
  cp $O/bench_$c.json $O/bench_${c}_$(date +%s).json
done
