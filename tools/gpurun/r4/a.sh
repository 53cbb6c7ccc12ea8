#!/bin/bash
# Round 4 first GPU pass: full GPU suite (new native account RPC devices, K1 host feature images),
# the driver's bench command, serving kernel stats, native open-loop curves for the account RPCs.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.log 2>&1
echo "gpu tests rc=$?" >> $O/status.txt
tail -3 $O/gpu_tests.log >> $O/status.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || { echo "bench rc=$?" >> $O/status.txt; exit 3; }
echo "bench ok" >> $O/status.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o serving -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/status.txt
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc ltv --open-loop --rates 50000,100000,200000,300000 \
  --seconds 4 --json-out $O/ltv_curve.json > $O/ltv_curve.log 2>&1
echo "ltv curve rc=$?" >> $O/status.txt
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc abuse --open-loop --rates 50000,100000,200000 \
  --seconds 4 --json-out $O/abuse_curve.json > $O/abuse_curve.log 2>&1
echo "abuse curve rc=$?" >> $O/status.txt
