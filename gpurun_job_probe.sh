#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_probe.py > gpurun_out/host_probe.log 2>&1 || exit 1
