#!/bin/bash
# Round 6 (re-entry): validation at HEAD - GPU suite, smoke, serving bench x2, engine_only for
# cfg3 / cfg4 / cfg5, cfg2 serving, serving kernel statistics.
set -o pipefail
O=gpurun_out/r6q
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
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2; do
  step srv_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$i.json
done
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
step cfg4_eng 300 python bench.py --config cfg4 --scope engine_only --steps 200 --warmup 20 --json-out $R/$O/cfg4_eng.json
step cfg5_eng 300 python bench.py --config cfg5 --scope engine_only --steps 20 --warmup 3 --json-out $R/$O/cfg5_eng.json
step cfg2 300 python bench.py --config cfg2 --steps 20 --warmup 5 --json-out $R/$O/cfg2.json
cd /tmp
step prof_srv 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_srv -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_srv.json
