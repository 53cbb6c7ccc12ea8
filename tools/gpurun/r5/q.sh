#!/bin/bash
# Round 5: per-batch post-state event ring + eight dedup regions -> pipeline depth is free up to 7.
# GPU engine / dp tests, then a same-box interleaved depth sweep (uniform serving, engine_only,
# Zipf 1.2 serving).
set -o pipefail
O=gpurun_out/r5q
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
step tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py tests/test_acct_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  for d in 3 4 5 6; do
    step srv_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --depth $d --json-out $R/$O/srv_d${d}_$i.json
    step eng_d${d}_$i 300 python bench.py --steps 300 --warmup 30 --depth $d --scope engine_only --json-out $R/$O/eng_d${d}_$i.json
    step zipf_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --depth $d --zipf 1.2 --json-out $R/$O/zipf_d${d}_$i.json
  done
done
