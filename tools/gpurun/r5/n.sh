#!/bin/bash
# Round 5: where the state queue's gaps come from - engine_only kernel timeline, and the serving
# run with the HIP runtime trace (launch call -> dispatch lead, tools/rocpd_timeline.py --api)
set -o pipefail
O=gpurun_out/r5n
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/eng -o eng -- \
  python $R/bench.py --steps 200 --warmup 30 --scope engine_only > $R/$O/eng.log 2>&1
rc=$?; echo "eng rc=$rc" >> $R/$O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/srv -o srv -- \
  python $R/bench.py --steps 3 --warmup 2 --rounds 4 > $R/$O/srv.log 2>&1
rc=$?; echo "srv rc=$rc" >> $R/$O/status.txt
exit $rc
