#!/bin/bash
# Round 4 final validation at HEAD: the whole GPU suite, smoke(), the driver's bench command
# (twice), engine_only, the Zipf serving runs, cfg4 / cfg5 fp32.
set -o pipefail
O=gpurun_out/r4v
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -3 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench1 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench1.json
step bench2 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench2.json
step engine 400 python bench.py --steps 20 --warmup 5 --scope engine_only --json-out $R/$O/engine.json
step zipf12 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json
step zipf105 400 python bench.py --steps 20 --warmup 5 --zipf 1.05 --json-out $R/$O/bench_zipf105.json
step cfg4 300 python bench.py --config cfg4 --steps 20 --warmup 5 --json-out $R/$O/cfg4.json
step cfg5 300 python bench.py --config cfg5 --steps 20 --warmup 5 --json-out $R/$O/cfg5.json
