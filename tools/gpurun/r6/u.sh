#!/bin/bash
# Round 6: K1 writes only the encoded FeatureVector chunks it filled (+ the length byte's chunk)
# to pinned host memory (B) vs the whole 128-byte image (A): same box, interleaved serving runs.
set -o pipefail
O=gpurun_out/r6u
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
SO=$R/igaming_platform_amd/_hipk.cpython-310-x86_64-linux-gnu.so
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2 3 4; do
  for v in A B; do
    cp $R/ab/_hipk_$v.so $SO
    step srv_${v}$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_${v}$i.json
  done
done
cp $R/ab/_hipk_B.so $SO
step tests 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "encoded or fenc or feature"
for i in 1 2; do
  step mixed_$i 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_$i.json
done
