#!/bin/bash
# Round 6: tree traversal from LDS (ds_read node tables, phased ILP), feature-major X tile: tree parity
# tests, standalone tree bench, engine_only and serving.
set -o pipefail
O=gpurun_out/r6l
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
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step tests 400 $T tests/test_trees_general_gpu.py tests/test_kernels_gpu.py
step tree 200 python tools/tree_bench.py
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
step srv 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv.json
step srv2 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv2.json
