#!/bin/bash
# Round 6: cached HLL estimates + routed exchange outputs + fused exchange insert; link index
# chunked; GPU suite, serving / SPMD / engine benches, mixed traffic, kernel statistics.
set -o pipefail
O=gpurun_out/r6d
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
  step plain_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/plain_$i.json
  IGP_BENCH_SPMD=1 step spmd_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_$i.json
done
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
cd /tmp
step prof_plain 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_plain -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_plain.json
IGP_BENCH_SPMD=1 step prof_spmd 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_spmd -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_spmd.json
