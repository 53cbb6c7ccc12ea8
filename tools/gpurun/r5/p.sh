#!/bin/bash
# Round 5: same-box interleaved A/B of the fused post-K1 update (IGP_UPD_FUSED=1) against the two
# launches (hot + multi), three times each, uniform serving / engine_only and Zipf(1.2) serving.
set -o pipefail
O=gpurun_out/r5p
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
for i in 1 2 3; do
  for f in 1 0; do
    export IGP_UPD_FUSED=$f
    step srv_f${f}_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_f${f}_$i.json
    step eng_f${f}_$i 300 python bench.py --steps 300 --warmup 30 --scope engine_only --json-out $R/$O/eng_f${f}_$i.json
    step zipf_f${f}_$i 300 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/zipf_f${f}_$i.json
  done
done
