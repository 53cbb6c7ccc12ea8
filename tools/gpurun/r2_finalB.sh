#!/bin/bash
# round-end validation B: request-path scopes (e2e, gRPC), cfg1 over gRPC, and the kernel trace
# of the default bench (last GPU step)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python bench.py --scope e2e --steps 200 --warmup 20 --json-out $O/scope_e2e.json > $O/scope_e2e.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scope grpc --rpc batch --json-out $O/scope_grpc_batch.json > $O/scope_grpc_batch.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --scope grpc --rpc tx --json-out $O/scope_grpc_tx.json > $O/scope_grpc_tx.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_cfg1.py > $O/bench_cfg1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/final -o run -- python bench.py --steps 100 --warmup 10 > $O/prof.log 2>&1 || exit 5
python tools/rocpd_stats.py /tmp/final/run_results.db > $O/cfg3_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/final/run_results.db --last 60 --skip-tail 5 > $O/cfg3_timeline.txt
