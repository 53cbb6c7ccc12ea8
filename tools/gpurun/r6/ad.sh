#!/bin/bash
# Round 6: serving over the pipeline depth (slots): a slot stays held while its caller copies
# the step's results and feature images out (release ~73 us per step, slot waits 1.2 per step at
# depth 4); depth 4 / 5 / 6 / 7 interleaved, 2 runs each; /dev/shm size of the box.
set -o pipefail
O=gpurun_out/r6ad
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
df -h /dev/shm > $R/$O/devshm.txt 2>&1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2; do
  for d in 4 5 6 7; do
    step srv_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --depth $d --json-out $R/$O/srv_d${d}_$i.json
  done
done
