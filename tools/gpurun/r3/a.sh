#!/bin/bash
# round 3, first GPU pass: GPU suite on the native serving core, default bench, e2e scope
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo "tests rc=$?" >> $O/status.txt
timeout -k 10 200 python bench.py --json-out $O/bench_default.json > $O/bench.log 2>&1 || exit 3
for t in 6 12; do
  timeout -k 10 300 python tools/bench_e2e.py --scope e2e --steps 300 --warmup 20 --threads $t --json-out $O/e2e_t$t.json > $O/e2e_t$t.log 2>&1 || exit 4
done
