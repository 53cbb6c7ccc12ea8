#!/bin/bash
# Round 6 final validation at HEAD: the driver's round-end steps (GPU suite, smoke, bench.py
# defaults) plus cfg4 / cfg5 through the account routers and mixed traffic.
set -o pipefail
O=gpurun_out/r6ar
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
step bench_default 400 python bench.py --json-out $R/$O/bench_default.json
step bench_20 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench_20.json
step cfg5 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5.json
step cfg4 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
