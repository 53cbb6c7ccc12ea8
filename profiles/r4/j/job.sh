#!/bin/bash
# Round 4: serving pipeline depth A/B (batches in flight per GPU), same box, uniform stream.
set -o pipefail
O=gpurun_out/r4j
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -1 $R/$O/$name.log | cut -c1-400 >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
for v in 3:0 4:0 3:1 4:1 3:0 4:0 3:1 4:1; do
  d=${v%:*}; export IGP_DEDUP_STATE=${v#*:}
  step bench_d${d}_ds$IGP_DEDUP_STATE 300 python bench.py --steps 40 --warmup 5 --depth $d \
    --json-out $R/$O/bench_d${d}_ds${IGP_DEDUP_STATE}_$RANDOM.json
done
export IGP_DEDUP_STATE=0
step engine_d3 300 python bench.py --steps 40 --warmup 5 --depth 3 --scope engine_only --json-out $R/$O/engine_d3.json
step engine_d4 300 python bench.py --steps 40 --warmup 5 --depth 4 --scope engine_only --json-out $R/$O/engine_d4.json
export IGP_DEDUP_STATE=1
step engine_d3_ds 300 python bench.py --steps 40 --warmup 5 --depth 3 --scope engine_only --json-out $R/$O/engine_d3_ds1.json
