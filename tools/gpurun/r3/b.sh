#!/bin/bash
# round 3, second GPU pass: GPU suite, serving-scope bench (default), engine-only bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo "tests rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --json-out $O/serving_default.json > $O/serving_default.log 2>&1 || exit 3
for t in 12 16; do
  timeout -k 10 300 python bench.py --threads $t --steps 600 --warmup 40 --json-out $O/serving_t$t.json > $O/serving_t$t.log 2>&1 || exit 4
done
timeout -k 10 200 python bench.py --scope engine_only --json-out $O/engine_only.json > $O/engine_only.log 2>&1 || exit 5
