#!/bin/bash
# Round 5 (end, tree groups at 256 workgroups): the whole GPU suite, smoke(), the driver bench, engine_only, exchange at world 1, cfg5 / cfg4.
set -o pipefail
O=gpurun_out/r5bh
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
step gpu_tests 1500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench.json
step engine 300 python bench.py --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/engine.json
IGP_BENCH_SPMD=1 step spmd 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd.json
step cfg5 400 python bench.py --config cfg5 --steps 20 --warmup 5 --json-out $R/$O/cfg5.json
step cfg4 400 python bench.py --config cfg4 --steps 20 --warmup 5 --json-out $R/$O/cfg4.json
