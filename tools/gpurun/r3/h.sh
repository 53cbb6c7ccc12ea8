#!/bin/bash
# round 3, pass h: full GPU suite, smoke, default bench; cfg4 weight-prefetch depth A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || exit 4
for pf in 2 5 2 5; do
  IGP_MC_PF=$pf timeout -k 10 200 python bench.py --config cfg4 --numerics bf16 --steps 400 --warmup 50 >> $O/cfg4_pf_ab.log 2>&1 || exit 5
  echo "pf=$pf $(tail -n 1 $O/cfg4_pf_ab.log | head -c 300)" >> $O/status.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run -- python bench.py --config cfg4 --numerics bf16 --steps 200 --warmup 30 > $O/prof_cfg4.log 2>&1 || exit 6
