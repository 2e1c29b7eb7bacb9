#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_nmprobe -o run --output-format csv -- python3 tools/nm_probe.py > gpurun_out/r3_nmprobe.log 2>&1 || exit $?
grep engine gpurun_out/r3_nmprobe.log
f=$(find gpurun_out/r3_nmprobe -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -12
find gpurun_out/r3_nmprobe -name '*kernel_trace.csv' -delete
