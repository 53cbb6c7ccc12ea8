#!/bin/bash
# Round 5 first pass at HEAD (hygiene + ADVICE fixes, multi-round serving step): the GPU suite,
# the driver's bench command (uniform / Zipf 1.2), K1 on cold batches with and without the
# single-event update, and the serving kernel stats.
set -o pipefail
O=gpurun_out/r5a
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
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step bench_zipf 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json
KB_K1_MODES=full,nodedup step kbench 300 python tools/kbench.py --cold --rounds 20
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o serving -- \
  python $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1
echo "prof rc=$?" >> $R/$O/status.txt
