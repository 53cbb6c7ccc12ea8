#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_stream.py > gpurun_out/dbg_s.log 2>&1
exit 0
