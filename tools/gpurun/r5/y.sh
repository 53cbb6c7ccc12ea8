#!/bin/bash
# Round 5: split GRU clusters with rcp gates, up to 256 rows, one abuse stream: trace, tests,
# CheckBonusAbuse curve, cfg5 bench through the account router.
set -o pipefail
O=gpurun_out/r5y
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
step trace 240 python tools/gru_wsx_trace.py --rows 256
step tests 500 python -u -m pytest tests/test_gru_gpu.py tests/test_acct_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for rate in 50000 100000 200000 300000 400000; do
  step abuse_$rate 300 python tools/host_profile.py --backend gpu --rpc abuse --rate $rate --seconds 3 --clients 8 --workers 8 --json-out $R/$O/abuse_$rate.json
done
step cfg5 400 python bench.py --config cfg5 --steps 20 --warmup 3 --json-out $R/$O/cfg5.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o p -- \
  python $R/tools/host_profile.py --backend gpu --rpc abuse --rate 100000 --seconds 2 --clients 8 --workers 8 > $R/$O/prof.log 2>&1)
echo "prof rc=$?" >> $R/$O/status.txt
