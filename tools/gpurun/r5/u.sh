#!/bin/bash
# Round 5: counter names available on gfx950 (for the tree_head PMC pass), and the serving depth
# sweep again after the K1 / slab changes.
set -o pipefail
O=gpurun_out/r5u
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/$O/list_avail.txt 2>&1
echo "list rc=$?" >> $R/$O/status.txt
cd $R
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
}
for i in 1 2; do
  for d in 4 5 6; do
    step srv_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --depth $d --json-out $R/$O/srv_d${d}_$i.json
  done
done
