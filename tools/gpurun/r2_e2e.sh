#!/bin/bash
# end-to-end scopes on 1 GPU after the host-path rework (AccountIndex 16-B entries + prefetch,
# arena parse, single-buffer serializer, async link index)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python tools/bench_e2e.py --scope e2e --threads 1 --steps 100 --warmup 10 > gpurun_out/r2/e2e_t1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --scope e2e --steps 300 --warmup 20 > gpurun_out/r2/e2e.log 2>&1 || exit 2
timeout -k 10 300 python tools/bench_e2e.py --scope e2e --threads 6 --steps 300 --warmup 20 > gpurun_out/r2/e2e_t6.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc batch --clients 8 --seconds 10 > gpurun_out/r2/grpc_batch.log 2>&1 || exit 4
