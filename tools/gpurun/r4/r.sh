#!/bin/bash
# round 4, pass r: hot-account apply cost vs rows of the account (tools/hot_apply_bench.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $R/$O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dedup_gpu.py tests/test_dp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/tests.log 2>&1 || { echo "tests rc=$?" >> $R/$O/status.txt; exit 1; }
OUT=$R/$O/hot_apply.json timeout -k 10 300 python tools/hot_apply_bench.py > $R/$O/hot_apply.log 2>&1
echo "hot_apply rc=$?" >> $R/$O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json > $R/$O/zipf12.log 2>&1
echo "zipf12 rc=$?" >> $R/$O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --zipf 1.05 --json-out $R/$O/bench_zipf105.json > $R/$O/zipf105.log 2>&1
echo "zipf105 rc=$?" >> $R/$O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench_uniform.json > $R/$O/uniform.log 2>&1
echo "uniform rc=$?" >> $R/$O/status.txt
