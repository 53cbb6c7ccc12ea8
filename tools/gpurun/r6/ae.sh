#!/bin/bash
# Round 6: validation at serving depth 6 - GPU suite (with the two-process exchange test), smoke,
# the driver's command x3, SPMD world 1, engine_only, mixed traffic x2.
set -o pipefail
O=gpurun_out/r6ae
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
done
IGP_BENCH_SPMD=1 step spmd 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd.json
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
for i in 1 2; do
  step mixed_$i 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed_$i.json
done
