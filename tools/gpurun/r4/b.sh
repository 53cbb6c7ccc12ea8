#!/bin/bash
# Round 4 second pass: account-RPC GPU tests, the open-loop tail probe, the serving bench under a
# uniform / Zipf account spread (128 distinct requests over 1 M accounts) + its kernel stats.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_acct_gpu.py -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/acct_gpu_tests.log 2>&1
echo "acct gpu tests rc=$?" >> $O/status.txt
timeout -k 10 200 python tools/acct_probe.py ltv 100000 4 > $O/probe_ltv_100k.log 2>&1; echo "probe ltv rc=$?" >> $O/status.txt
timeout -k 10 200 python tools/acct_probe.py ltv 200000 4 > $O/probe_ltv_200k.log 2>&1; echo "probe ltv2 rc=$?" >> $O/status.txt
timeout -k 10 200 python tools/acct_probe.py abuse 150000 4 > $O/probe_abuse_150k.log 2>&1; echo "probe abuse rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out $O/bench_uniform.json > $O/bench_uniform.log 2>&1
echo "bench uniform rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $O/bench_zipf.json > $O/bench_zipf.log 2>&1
echo "bench zipf rc=$?" >> $O/status.txt
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o serving_uniform -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/status.txt
