#!/bin/bash
# Round 4: five-region dedup ring; serving / engine_only at pipeline depth 3 vs 4 (same box) +
# the device-pipeline GPU tests.
set -o pipefail
O=gpurun_out/r4l
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -2 $R/$O/$name.log | cut -c1-300 >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dedup_gpu.py tests/test_dp_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider
for d in 3 4 3 4; do
  step bench_d$d 300 python bench.py --steps 40 --warmup 5 --depth $d --json-out $R/$O/bench_d${d}_$RANDOM.json
  step engine_d$d 300 python bench.py --steps 40 --warmup 5 --depth $d --scope engine_only --json-out $R/$O/engine_d${d}_$RANDOM.json
done
