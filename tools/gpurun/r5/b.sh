#!/bin/bash
# Round 5: K1 attribution - kernel time on cold rotating batches with parts of K1 skipped
# (AssembleArgs.ablate bits: 1 HLL, 2 dedup+update, 4 blacklist/ip, 8 amounts, 16 ext, 32 ts ring,
# 64 rt+batch, 128 output stores, 512 = feature images to pinned host memory as in serving)
set -o pipefail
O=gpurun_out/r5c
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
KB_K1_MODES=full KB_ABLATE=0,512,1,2,4,8,16,32,64,128,125,253,255,0 timeout -k 10 300 python tools/kbench.py --cold --rounds 10 > $R/$O/kbench.log 2>&1
echo "kbench rc=$?" >> $R/$O/status.txt
