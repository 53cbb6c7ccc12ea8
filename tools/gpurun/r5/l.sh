#!/bin/bash
# Round 5: K1 with its arguments read by vector loads (kernarg_vgpr) and HIP_FORCE_DEV_KERNARG=1:
# K1 alone on cold batches, the driver's bench command, engine_only, serving kernel stats.
set -o pipefail
O=gpurun_out/r5l
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
KB_K1_MODES=- KB_ABLATE=0,512,255 step kbench 300 python tools/kbench.py --cold --rounds 10
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step engine 400 python bench.py --steps 300 --warmup 30 --scope engine_only --json-out $R/$O/engine.json
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o serving -- \
  python $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1)
echo "prof rc=$?" >> $R/$O/status.txt
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_acct_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $R/$O/gpu_tests.log 2>&1
echo "gpu tests rc=$?" >> $R/$O/status.txt
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $R/$O/dp_tests.log 2>&1
echo "dp tests rc=$?" >> $R/$O/status.txt
