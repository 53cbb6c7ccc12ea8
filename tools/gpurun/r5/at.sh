#!/bin/bash
# Round 5: after removing the serial mode and the asynchronous issue thread: engine / dp GPU tests, bench.
set -o pipefail
O=gpurun_out/r5at
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
step gpu_tests 900 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py tests/test_dedup_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step engine 300 python bench.py --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/engine.json
