#!/bin/bash
# GPU suite + smoke + default bench at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 200 python bench.py --json-out $O/bench_default.json > $O/bench.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --config cfg2 --json-out $O/bench_cfg2.json >> $O/bench.log 2>&1 || exit 4
