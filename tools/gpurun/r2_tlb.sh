#!/bin/bash
# K1 address translation: UTCL1 hit / miss / request counters (one PMC pass, 4 TCP counters),
# then TA busy vs SQ wave cycles; the counter list of this GPU first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tlb
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
IGP_ROCTX=0 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum --kernel-include-regex "feature_assemble|tree_kernel|mlp_head" --output-format csv -d /tmp/tlb -o run -- python bench.py --steps 30 --warmup 5 > $O/pmc.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/tlb > $O/pmc_tlb.txt
exit $rc
