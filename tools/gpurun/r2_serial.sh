#!/bin/bash
# serial single-stream mode for small micro-batches: parity tests, then cfg2 A/B (3 passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2serial
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_serial.log 2>&1 || exit 1
for pass in 1 2 3; do
  for x in 0 2048; do
    IGP_SERIAL_MAX_BUCKET=$x timeout -k 10 200 python bench.py --config cfg2 --steps 400 --warmup 40 --json-out $O/cfg2_s${x}_$pass.json > $O/cfg2_s${x}_$pass.log 2>&1 || exit 2
  done
done
for x in 0 16384; do
  IGP_SERIAL_MAX_BUCKET=$x timeout -k 10 200 python bench.py --steps 400 --warmup 40 --json-out $O/cfg3_s${x}.json > $O/cfg3_s${x}.log 2>&1 || exit 3
done
