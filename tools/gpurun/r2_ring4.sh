#!/bin/bash
# four-region dedup ring, the copy stage's region wait skipped when the host sees it complete:
# GPU suite, then a same-box A/B against always queueing the wait (IGP_DEDUP_QUERY=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ring4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for i in 1 2; do
  for q in 1 0; do
    IGP_DEDUP_QUERY=$q timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --json-out $O/cfg3_q${q}_$i.json > $O/cfg3_q${q}_$i.log 2>&1 || exit 3
    IGP_DEDUP_QUERY=$q timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --json-out $O/cfg2_q${q}_$i.json > $O/cfg2_q${q}_$i.log 2>&1 || exit 4
  done
done
