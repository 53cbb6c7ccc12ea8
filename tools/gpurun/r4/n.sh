#!/bin/bash
# 16-wave split GRU as the default at H = 256: GRU / abuse / account GPU tests, then cfg5 bench
# (fp32 split, per-slot streams) and the serving-rank shape (one stream) from the sweep tool.
set -o pipefail
O=gpurun_out/r4n
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -3 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step gru_tests 600 python -u -m pytest tests/test_gru_gpu.py tests/test_acct_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  step cfg5_fp32_$i 300 python bench.py --config cfg5 --steps 20 --warmup 5 --json-out $R/$O/cfg5_fp32_$i.json
done
step cfg5_bf16 300 python bench.py --config cfg5 --numerics bf16 --steps 20 --warmup 5 --json-out $R/$O/cfg5_bf16.json
OUT=$R/$O/gru_x3_sweep.json step gru_x3 300 python tools/gru_x3_bench.py
