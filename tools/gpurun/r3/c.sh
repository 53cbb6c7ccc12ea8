#!/bin/bash
# round 3, third GPU pass: GPU suite, serving bench, unary gRPC offered-load curve, ScoreBatch over gRPC, rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo "tests rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --json-out $O/serving_default.json > $O/serving_default.log 2>&1 || exit 3
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc tx --open-loop --clients 10 --seconds 4 --rates 10000,25000,50000,75000,100000,150000 --json-out $O/grpc_tx_curve.json > $O/grpc_tx_curve.log 2>&1 || exit 4
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc batch --clients 8 --json-out $O/grpc_batch.json > $O/grpc_batch.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rs -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 300 --warmup 30 > $GRAFT_REPO_ROOT/$O/prof_serving.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python tools/rocpd_stats.py /tmp/rs/run_results.db > $O/serving_kernel_stats.txt
