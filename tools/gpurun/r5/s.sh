#!/bin/bash
# Round 5: dedup insert reads the batch from the pinned slab (no H2D copy per batch).
set -o pipefail
O=gpurun_out/r5s
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
KB_VARIANTS=0,512 KB_TRACE_OUT=$R/$O/k1trace step kbench 300 python tools/kbench.py --cold --rounds 10
for i in 1 2; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
  step eng_$i 300 python bench.py --steps 300 --warmup 30 --scope engine_only --json-out $R/$O/eng_$i.json
  step zipf_$i 300 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/zipf_$i.json
  step zipf105_$i 300 python bench.py --steps 20 --warmup 5 --zipf 1.05 --json-out $R/$O/zipf105_$i.json
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- \
  python $R/bench.py --steps 5 --warmup 3 --rounds 8 > $R/$O/prof.log 2>&1)
rc=$?; echo "prof rc=$rc" >> $R/$O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
step cfg5 400 python bench.py --config cfg5 --steps 20 --warmup 3 --json-out $R/$O/cfg5.json
step cfg4 400 python bench.py --config cfg4 --steps 20 --warmup 3 --json-out $R/$O/cfg4.json
