#!/bin/bash
# cfg4 fused chain re-measure; cold RPCs: batched engine calls and micro-batched unary gRPC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/t_mlp.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config cfg4 --steps 300 --warmup 30 > gpurun_out/r2/bench_cfg4_fused.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof4 -o run -- python bench.py --config cfg4 --steps 100 --warmup 10 > gpurun_out/r2/prof4.log 2>&1
python tools/rocpd_stats.py /tmp/prof4/run_results.db > gpurun_out/r2/cfg4_fused_kernel_stats.txt
timeout -k 10 300 python tools/bench_e2e.py --scope engine_batched --rpc ltv --accounts 65536 --steps 50 > gpurun_out/r2/cold_engine_ltv.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_e2e.py --scope engine_batched --rpc abuse --accounts 65536 --steps 30 > gpurun_out/r2/cold_engine_abuse.log 2>&1 || exit 4
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc ltv --accounts 65536 --clients 16 --seconds 8 > gpurun_out/r2/cold_grpc_ltv.log 2>&1 || exit 5
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc abuse --accounts 65536 --clients 16 --seconds 8 > gpurun_out/r2/cold_grpc_abuse.log 2>&1 || exit 6
