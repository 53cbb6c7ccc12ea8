#!/bin/bash
# round 3, pass f: GRU direction / layout lowering + exchange stream-map tests, default serving bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gru_gpu.py tests/test_dp_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --scope e2e --json-out $O/e2e.json > $O/e2e.log 2>&1 || exit 4
