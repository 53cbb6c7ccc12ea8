#!/bin/bash
# round 3, pass d: split-precision MLP chain / GRU tests + cfg4 / cfg5 benches (fp32 default, bf16 alongside),
# unary gRPC curve at lower offered loads
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mlp_fused_gpu.py tests/test_gru_gpu.py tests/test_engine_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2  # timeout / abort / fault: nothing more on the GPU
for c in cfg4 cfg5; do
  for nm in fp32 bf16; do
    timeout -k 10 300 python bench.py --config $c --numerics $nm --steps 300 --warmup 30 --json-out $O/bench_${c}_$nm.json > $O/bench_${c}_$nm.log 2>&1 || exit 3
  done
done
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc tx --open-loop --clients 8 --seconds 4 --json-out $O/grpc_tx_curve.json > $O/grpc_tx_curve.log 2>&1 || exit 4
