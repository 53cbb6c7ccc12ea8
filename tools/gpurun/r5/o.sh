#!/bin/bash
# Round 5: update_multi regressed 10 -> 22 us since r5a. A/B of device-resident kernel arguments
# (HIP_FORCE_DEV_KERNARG) x one fused post-K1 update launch (IGP_UPD_FUSED), bench + kernel stats.
set -o pipefail
O=gpurun_out/r5o
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
step tests 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "hot or multi or reads_see or segment"
for kf in 11 01 10 00; do
  k=${kf:0:1}; f=${kf:1:1}
  export HIP_FORCE_DEV_KERNARG=$k IGP_UPD_FUSED=$f
  step srv_$kf 300 python bench.py --steps 20 --warmup 5 --json-out $R/$O/srv_$kf.json
  step eng_$kf 300 python bench.py --steps 300 --warmup 30 --scope engine_only --json-out $R/$O/eng_$kf.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$kf -o p -- \
    python $R/bench.py --steps 5 --warmup 3 --rounds 8 > $R/$O/prof_$kf.log 2>&1)
  rc=$?; echo "prof_$kf rc=$rc" >> $R/$O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
