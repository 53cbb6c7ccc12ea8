#!/bin/bash
# Round 6: account-RPC benches with the sink-based multi-thread driver (cfg4 / cfg5 serving),
# cfg5 engine sweep (depth, split-GRU tile rows), cfg1 (CPU backend) and the unary
# ScoreTransaction saturation curve, cfg2 serving.
set -o pipefail
O=gpurun_out/r6e
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for t in 1 4; do
  step cfg5_srv_t$t 400 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads $t --json-out $R/$O/cfg5_srv_t$t.json
  step cfg4_srv_t$t 400 python bench.py --config cfg4 --steps 5 --warmup 1 --drive-threads $t --json-out $R/$O/cfg4_srv_t$t.json
done
step cfg5_srv_t4b 400 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 4 --json-out $R/$O/cfg5_srv_t4b.json
step cfg5_srv_t8 400 python bench.py --config cfg5 --steps 5 --warmup 1 --drive-threads 8 --json-out $R/$O/cfg5_srv_t8.json
for d in 2 3; do
  for r in 16 32; do
    IGP_GRU_X3_ROWS=$r step cfg5_eng_d${d}_r$r 300 python bench.py --config cfg5 --scope engine_only --depth $d --steps 20 --warmup 3 --json-out $R/$O/cfg5_eng_d${d}_r$r.json
  done
done
step cfg4_eng 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_eng.json
step cfg2 300 python bench.py --config cfg2 --steps 20 --warmup 5 --json-out $R/$O/cfg2.json
step cfg1_curve 600 python -u tools/bench_e2e.py --scope grpc --rpc tx --open-loop --backend cpu --model cfg1 --rates 50000,100000,150000,200000,250000 --seconds 4 --clients 8 --json-out $R/$O/cfg1_curve.json
step tx_curve 600 python -u tools/bench_e2e.py --scope grpc --rpc tx --open-loop --rates 600000,800000,1000000,1200000 --seconds 4 --clients 8 --json-out $R/$O/tx_curve.json
