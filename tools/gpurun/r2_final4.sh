#!/bin/bash
# re-created container: rebuilt .so files checked on the GPU (suite, smoke, default + cfg2/cfg4/cfg5 benches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 200 python bench.py --json-out $O/bench_default.json >> $O/bench.log 2>&1 || exit 3
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 2000 --warmup 100 --json-out $O/bench_$c.json >> $O/bench.log 2>&1 || exit 4
done
