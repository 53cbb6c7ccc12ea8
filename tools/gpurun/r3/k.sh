#!/bin/bash
# round 3, pass k: two-clusters-per-CU GRU (ws=3) parity + A/B vs ws=1, phase traces, cfg5 bench A/B;
# then the round-end tiers (full GPU suite, smoke, default bench) and the native gRPC curves
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $O/gru_tests.txt 2>&1
rc=$?; echo "gru tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
GRU_WS_ONLY=1 GRU_BATCHES=4096,2048,512 OUT=$O/gru_sweep.json timeout -k 10 200 python tools/gru_bench.py > $O/gru_sweep.log 2>&1 || exit 3
for w in 1 3; do timeout -k 10 120 python tools/gru_ws_trace.py 4096 $w > $O/gru_trace_ws$w.txt 2>&1 || exit 4; done
for w in 1 3 1 3; do
  IGP_GRU_WS_MODE=$w timeout -k 10 200 python bench.py --config cfg5 --numerics bf16 --steps 100 --warmup 10 --json-out $O/cfg5_bf16_ws$w.json >> $O/cfg5_ab.log 2>&1 || exit 5
  echo "ws=$w $(tail -c 250 $O/cfg5_bf16_ws$w.json)" >> $O/status.txt
done
for cfg in "32 5" "64 5" "64 3" "32 5" "64 5" "64 3"; do
  set -- $cfg
  IGP_MLP_ROWS=$1 IGP_MC_PF=$2 timeout -k 10 200 python bench.py --config cfg4 --numerics bf16 --steps 400 --warmup 50 --json-out $O/cfg4_r$1_pf$2.json >> $O/cfg4_ab.log 2>&1 || exit 11
  echo "cfg4 rows=$1 pf=$2 $(tail -c 200 $O/cfg4_r$1_pf$2.json)" >> $O/status.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 6
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 7
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 8
echo "bench $(tail -c 300 $O/bench_default.json)" >> $O/status.txt
timeout -k 10 400 python tools/bench_e2e.py --scope grpc --rpc tx --open-loop --clients 8 --seconds 4 --rates 10000,50000,100000,200000,400000 --json-out $O/grpc_tx_native_curve.json > $O/grpc_tx_native_curve.log 2>&1 || exit 9
timeout -k 10 300 python tools/bench_e2e.py --scope grpc --rpc batch --clients 8 --seconds 8 --json-out $O/grpc_batch_native.json > $O/grpc_batch_native.log 2>&1 || exit 10
