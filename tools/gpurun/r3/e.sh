#!/bin/bash
# round 3, pass e: one-launch cfg3 (tree -> head -> K5) equivalence + A/B, engine GPU tests alone,
# cfg4 / cfg5 fp32 + bf16 engine benches, unary gRPC curve
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
for th in 0 1 0 1; do
  IGP_TREE_HEAD=$th timeout -k 10 200 python bench.py --config cfg3 --scope engine_only --steps 400 --warmup 50 --json-out $O/cfg3_engine_th$th.json >> $O/cfg3_ab.log 2>&1 || exit 3
  echo "th=$th $(tail -c 400 $O/cfg3_engine_th$th.json)" >> $O/status.txt
done
IGP_TREE_HEAD=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_th1 -o run -- python bench.py --config cfg3 --scope engine_only --steps 200 --warmup 30 > $O/prof_th1.log 2>&1 || exit 4
for c in cfg4 cfg5; do
  for nm in fp32 bf16; do
    timeout -k 10 300 python bench.py --config $c --numerics $nm --steps 300 --warmup 30 --json-out $O/bench_${c}_$nm.json > $O/bench_${c}_$nm.log 2>&1 || exit 5
  done
done
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc tx --open-loop --clients 8 --seconds 4 --json-out $O/grpc_tx_curve.json > $O/grpc_tx_curve.log 2>&1 || exit 6
