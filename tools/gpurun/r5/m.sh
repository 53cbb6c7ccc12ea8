#!/bin/bash
# Round 5 second measured pass: the GPU suite (state clock, RCCL teardown, hot-account kernel),
# K1 alone, the driver's bench command (uniform / Zipf 1.2), engine_only, serving kernel stats.
set -o pipefail
O=gpurun_out/r5m
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step engine_tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_acct_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step dp_tests 400 python -u -m pytest tests/test_dp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
KB_K1_MODES=- KB_ABLATE=0,512,255 step kbench 300 python tools/kbench.py --cold --rounds 10
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step bench_zipf 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json
step engine 400 python bench.py --steps 300 --warmup 30 --scope engine_only --json-out $R/$O/engine.json
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o serving -- \
  python $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1)
echo "prof rc=$?" >> $R/$O/status.txt
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/profz -o zipf -- \
  python $R/bench.py --steps 20 --warmup 5 --zipf 1.2 > $R/$O/profz.log 2>&1)
echo "profz rc=$?" >> $R/$O/status.txt
