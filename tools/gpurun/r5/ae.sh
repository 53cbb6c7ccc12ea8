#!/bin/bash
# Round 5: the exchange serving path at N = 1 with the HIP runtime trace (host issue times).
set -o pipefail
O=gpurun_out/r5ae
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
IGP_BENCH_SPMD=1 IGP_XCHG_RESULTS=d2h timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof -o p -- \
  python $R/bench.py --steps 3 --warmup 2 --rounds 8 > $R/$O/prof.log 2>&1
echo "prof rc=$?" >> $R/$O/status.txt
