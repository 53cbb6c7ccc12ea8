#!/bin/bash
# Round 5: kernel timeline of the exchange serving path at N = 1; cfg4 engine_only A/B of
# device-resident kernel arguments.
set -o pipefail
O=gpurun_out/r5ab
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
HIP_FORCE_DEV_KERNARG=0 step cfg4_k0 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_k0.json
HIP_FORCE_DEV_KERNARG=1 step cfg4_k1 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_k1.json
(cd /tmp && IGP_BENCH_SPMD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- \
  python $R/bench.py --steps 3 --warmup 2 --rounds 8 > $R/$O/prof.log 2>&1)
echo "prof rc=$?" >> $R/$O/status.txt
