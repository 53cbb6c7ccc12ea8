#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/gather_probe 1048576 > gpurun_out/gather_probe.log 2>&1 || exit 1
timeout -k 10 120 ./tools/probe/gather_probe 65536 >> gpurun_out/gather_probe.log 2>&1 || exit 2
