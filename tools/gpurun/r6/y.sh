#!/bin/bash
# Round 6: answers read known account ids back from the index (no per-call id copy): GPU suite,
# smoke, cfg4 x3, cfg5.
set -o pipefail
O=gpurun_out/r6y
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
for i in 1 2 3; do
  IGP_BENCH_THREADS_OUT=$R/$O/cfg4_${i}_threads.json step cfg4_$i 300 python bench.py --config cfg4 --steps 5 --warmup 1 --json-out $R/$O/cfg4_$i.json
done
step cfg5 300 python bench.py --config cfg5 --steps 5 --warmup 1 --json-out $R/$O/cfg5.json
