#!/bin/bash
# K1 vs trees vs head: UTCL1 stall counters (one PMC pass, 4 TCP counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tlb2
mkdir -p $O
IGP_ROCTX=0 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum --kernel-include-regex "feature_assemble|tree_kernel|mlp_head" --output-format csv -d /tmp/tlb2 -o run -- python bench.py --steps 30 --warmup 5 > $O/pmc.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/tlb2 > $O/pmc_tlb_stalls.txt
[ $rc -eq 0 ] || exit $rc
IGP_ROCTX=0 timeout -s KILL 120 rocprofv3 --pmc TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_GATE_EN1_sum TCP_CLIENT_UTCL1_INFLIGHT_sum --kernel-include-regex "feature_assemble|tree_kernel|mlp_head" --output-format csv -d /tmp/tlb3 -o run -- python bench.py --steps 30 --warmup 5 > $O/pmc3.log 2>&1
rc=$?
python tools/pmc_summary.py /tmp/tlb3 > $O/pmc_tcp_cycles.txt
exit $rc
