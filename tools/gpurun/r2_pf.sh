#!/bin/bash
# dedup insert prefetch of the accounts' ring / HLL / RT lines (IGP_K1_PREFETCH): parity test,
# same-box A/B of cfg3 (x3 alternating) and cfg2, kernel trace with prefetch on
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pf
mkdir -p $O
IGP_K1_PREFETCH=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_dedup_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
for i in 1 2 3; do
  for p in 1 0; do
    IGP_K1_PREFETCH=$p timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_pf${p}_$i.json > $O/cfg3_pf${p}_$i.log 2>&1 || exit 2
  done
done
for p in 1 0; do
  IGP_K1_PREFETCH=$p timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --json-out $O/cfg2_pf${p}.json > $O/cfg2_pf${p}.log 2>&1 || exit 3
done
IGP_K1_PREFETCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pf -o run -- python bench.py --steps 300 --warmup 30 > $O/prof.log 2>&1 || exit 4
python tools/rocpd_stats.py /tmp/pf/run_results.db > $O/cfg3_pf1_kernel_stats.txt
python tools/rocpd_timeline.py /tmp/pf/run_results.db --last 40 --skip-tail 5 > $O/cfg3_pf1_timeline.txt
