#!/bin/bash
# Round 4 fifth pass: IGP_K1_PREFETCH A/B under the uniform serving stream (cold accounts),
# bench + kernel stats for each setting on the same box.
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -2 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
for pf in 0 1 0 1; do
  export IGP_K1_PREFETCH=$pf
  step bench_pf$pf 400 python bench.py --steps 40 --warmup 5 --json-out $R/$O/bench_pf${pf}_$RANDOM.json
done
cd /tmp
for pf in 0 1; do
  export IGP_K1_PREFETCH=$pf
  step prof_pf$pf 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_pf$pf -o s -- python $R/bench.py --steps 20 --warmup 5
done
