#!/bin/bash
# Round 6: exchange rows through the node-shared rows region (IGP_XCHG_ROWS=shm) - DP GPU tests,
# SPMD world-1 serving bench shm vs rccl vs plain; 1h-sum sliding vs compat A/B (the amount-ring
# reads of K1); mixed traffic; kernel traces with queue ids.
set -o pipefail
O=gpurun_out/r6c
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
for i in 1 2; do
  IGP_BENCH_SPMD=1 step spmd_shm_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_shm_$i.json
  IGP_BENCH_SPMD=1 IGP_XCHG_ROWS=rccl step spmd_rccl_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/spmd_rccl_$i.json
  step plain_$i 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/plain_$i.json
  step plain_compat_$i 300 python bench.py --steps 20 --warmup 5 --sum-mode compat --json-out $R/$O/plain_compat_$i.json
done
step eng 300 python bench.py --scope engine_only --steps 400 --warmup 20 --json-out $R/$O/eng.json
step eng_compat 300 python bench.py --scope engine_only --steps 400 --warmup 20 --sum-mode compat --json-out $R/$O/eng_compat.json
step mixed 400 python tools/bench_mixed.py --seconds 5 --json-out $R/$O/mixed.json
cd /tmp
IGP_BENCH_SPMD=1 step prof_shm 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_shm -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_shm.json
IGP_BENCH_SPMD=1 IGP_XCHG_ROWS=rccl step prof_rccl 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_rccl -o run -- python $R/bench.py --steps 10 --warmup 3 --json-out $R/$O/prof_rccl.json
