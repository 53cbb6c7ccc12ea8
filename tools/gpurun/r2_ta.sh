#!/bin/bash
# K1: is the texture-address (TA) path the limit? PMC on K1 alone (kbench)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ta
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" $O/avail.txt | sort -u > $O/ta_td_tcp.txt
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "feature_assemble" --output-format csv -d /tmp/ta1 -o run -- python tools/kbench.py --rounds 4 --only feature_assemble_no_update > $O/pmc1.log 2>&1
python tools/pmc_summary.py /tmp/ta1 --batch 8192 > $O/pmc_ta1.txt
