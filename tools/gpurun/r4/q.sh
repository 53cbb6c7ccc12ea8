#!/bin/bash
# round 4, pass q: hot accounts' multi-event apply with batched scan loads and LDS-resident HLL
# registers: engine / dedup / DP GPU tests, then the Zipf(1.2) and Zipf(1.05) serving benches
# and the Zipf(1.2) kernel stats (compare r4/p: update_multi_kernel 412.5 us per call)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4q
mkdir -p $R/$O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/$O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $R/$O/status.txt; tail -3 $R/$O/$name.log >> $R/$O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  [ $rc -eq 0 ] || exit $rc
  return 0
}
step tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dedup_gpu.py tests/test_dp_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step zipf12 400 python bench.py --steps 20 --warmup 5 --zipf 1.2 --json-out $R/$O/bench_zipf.json
step zipf105 400 python bench.py --steps 20 --warmup 5 --zipf 1.05 --json-out $R/$O/bench_zipf105.json
step uniform 400 python bench.py --steps 20 --warmup 5 --json-out $R/$O/bench_uniform.json
cd /tmp
step zprof 400 rocprofv3 --kernel-trace --stats -d /tmp/zprof -o zipf -- python $R/bench.py --steps 20 --warmup 5 --zipf 1.2
DB=$(ls /tmp/zprof/*/zipf_results.db /tmp/zprof/zipf_results.db 2>/dev/null | head -1)
python $R/tools/rocpd_stats.py "$DB" --top 25 > $R/$O/zipf_kernel_stats.txt 2>&1
