#!/bin/bash
# Round 6: tree-group target 384 workgroups (3 groups at 8192 rows) - GPU suite, then the
# driver's serving command and engine_only at 3 groups (default) vs 2 (forced), interleaved.
set -o pipefail
O=gpurun_out/r6am
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
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
for i in 1 2 3; do
  IGP_TREE_GROUPS=2 step srv_g2_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_g2_$i.json
  step srv_g3_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_g3_$i.json
done
for i in 1 2; do
  IGP_TREE_GROUPS=2 step eng_g2_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_g2_$i.json
  step eng_g3_$i 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng_g3_$i.json
done
