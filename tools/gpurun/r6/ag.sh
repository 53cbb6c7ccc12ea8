#!/bin/bash
# Round 6: tree node tables staged global -> LDS with global_load_lds (B) vs through registers
# (A): tree parity tests, standalone tree bench, engine_only and serving interleaved.
set -o pipefail
O=gpurun_out/r6ag
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
H=$R/igaming_platform_amd/_hipk.cpython-310-x86_64-linux-gnu.so
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
cp $R/ab/_hipk_B.so $H
step tests 500 python -u -m pytest tests/test_trees_general_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 150 --timeout-method thread
for v in A B; do
  cp $R/ab/_hipk_$v.so $H
  step tree_$v 200 python tools/tree_bench.py
done
for i in 1 2; do
  for v in A B; do
    cp $R/ab/_hipk_$v.so $H
    step eng_${v}$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_${v}$i.json
    step srv_${v}$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_${v}$i.json
  done
done
cp $R/ab/_hipk_B.so $H
