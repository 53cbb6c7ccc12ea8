#!/bin/bash
# round 4, pass x: the hot-account GPU tests (many devices / ips per hot account)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4x
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -k "hot_accounts" -v --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/tests.log 2>&1
echo "tests rc=$?" >> $R/$O/status.txt
