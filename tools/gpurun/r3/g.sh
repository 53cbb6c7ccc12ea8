#!/bin/bash
# round 3, pass g: full GPU suite, smoke, default bench (the driver's round-end tiers)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 4
