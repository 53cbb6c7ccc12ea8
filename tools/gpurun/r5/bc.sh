#!/bin/bash
# Round 5 (experiment): dedup insert reading the pinned slab (default) vs an H2D copy first.
set -o pipefail
O=gpurun_out/r5bc
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
step parity 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "direct_launch"
for i in 1 2 3; do
  step eng_slab_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_slab_$i.json
  IGP_AB_DEDUP_DEV=1 step eng_dev_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_dev_$i.json
done
for i in 1 2 3; do
  step srv_slab_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_slab_$i.json
  IGP_AB_DEDUP_DEV=1 step srv_dev_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_dev_$i.json
done
