#!/bin/bash
# round 3, pass j (re-created container, rebuilt .so): full GPU suite, smoke, default bench,
# native gRPC server curves (unary open loop, ScoreBatch), serving-scope kernel statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 4
echo "bench $(tail -c 300 $O/bench_default.json)" >> $O/status.txt
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc tx --open-loop --clients 8 --seconds 4 --rates 10000,50000,100000,200000,400000 --json-out $O/grpc_tx_native_curve.json > $O/grpc_tx_native_curve.log 2>&1 || exit 5
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc batch --clients 8 --seconds 8 --json-out $O/grpc_batch_native.json > $O/grpc_batch_native.log 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rs -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 300 --warmup 30 > $GRAFT_REPO_ROOT/$O/prof_serving.log 2>&1 || exit 7
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/rs/run_results.db > $O/serving_kernel_stats.txt
