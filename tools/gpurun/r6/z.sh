#!/bin/bash
# Round 6: (1) answers reading known account ids from the index (native B) vs a per-call id copy
# (A), cfg4 through the router, interleaved; (2) the split LTV chain's weight prefetch 2 k-steps
# ahead (P2) vs 1 (P1): chain kernel alone, cfg4 engine_only, the chain's GPU tests.
set -o pipefail
O=gpurun_out/r6z
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
N=$R/igaming_platform_amd/_native.cpython-310-x86_64-linux-gnu.so
H=$R/igaming_platform_amd/_hipk.cpython-310-x86_64-linux-gnu.so
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
cp $R/ab/_hipk_P1.so $H
for i in 1 2 3; do
  for v in A B; do
    cp $R/ab/_native_$v.so $N
    step cfg4_${v}$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_${v}$i.json
  done
done
cp $R/ab/_native_B.so $N
for i in 1 2; do
  for p in P1 P2; do
    cp $R/ab/_hipk_$p.so $H
    SPLIT=1 OUT=$R/$O/mlp_${p}_$i.json step mlp_${p}_$i 300 python tools/mlp_bench.py 8192
    step eng4_${p}_$i 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/eng4_${p}_$i.json
  done
done
step tests 300 python -u -m pytest tests/test_mlp_fused_gpu.py -x -v --timeout 120 --timeout-method thread
