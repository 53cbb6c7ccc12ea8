#!/bin/bash
# Round 4 sixth pass: cfg4 fused chain vs layer-wise large-tile GEMMs.
set -o pipefail
O=gpurun_out/r4f
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -4 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step tests 300 python -u -m pytest tests/test_mlp_fused_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider
export OUT=$R/$O/mlp_layerwise.json
step trace 200 python tools/mlp_layerwise_bench.py 8192 --trace
step layerwise 300 python tools/mlp_layerwise_bench.py 8192,16384
cd /tmp
export OUT=/tmp/lw.json
step prof 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o lw -- python $R/tools/mlp_layerwise_bench.py 8192
