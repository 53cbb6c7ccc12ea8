#!/bin/bash
# round 4, pass z: the many-devices hot-account test alone, then after the tests that precede it
# in the full suite (it failed once there)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4z
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "many_devices" -v --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/alone.log 2>&1
echo "alone rc=$?" >> $R/$O/status.txt
timeout -k 10 500 python -u -m pytest tests/test_acct_gpu.py tests/test_dedup_gpu.py tests/test_dp_gpu.py tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/seq.log 2>&1
echo "seq rc=$?" >> $R/$O/status.txt
