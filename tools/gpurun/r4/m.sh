#!/bin/bash
# Round 4 validation at HEAD (per-slot streams in the account devices, router pause/resume,
# layer-wise LTV test): the GPU suite, smoke(), the driver's bench command, engine_only; then
# the cfg5 f32-faithful GRU tile / concurrency sweep.
set -o pipefail
O=gpurun_out/r4m
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
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step engine 400 python bench.py --steps 20 --warmup 5 --scope engine_only --json-out $R/$O/engine.json
OUT=$R/$O/gru_x3_sweep.json step gru_x3 300 python tools/gru_x3_bench.py
# cfg4 chain: 8 vs 16 waves per 64-row workgroup, interleaved, fp32 (split) and bf16
for i in 1 2; do
  for w in 8 16; do
    IGP_MLP_WAVES=$w step cfg4_fp32_w${w}_$i 300 python bench.py --config cfg4 --steps 20 --warmup 5 --json-out $R/$O/cfg4_fp32_w${w}_$i.json
  done
done
for w in 8 16; do
  IGP_MLP_WAVES=$w step cfg4_bf16_w$w 300 python bench.py --config cfg4 --numerics bf16 --steps 20 --warmup 5 --json-out $R/$O/cfg4_bf16_w$w.json
done
