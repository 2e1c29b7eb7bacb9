#!/bin/bash
# round-2: one rank's share of the multi-GPU 3-D runs (eager vs graph-captured chunks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-share}
mkdir -p $O
timeout -k 10 300 python3 tools/bench3d.py --size 512 --dtype f32 --rank-of 4 --steps 40 > $O/c4_of4.log 2>&1 || { echo C4_FAILED; tail -20 $O/c4_of4.log; exit 1; }
tail -1 $O/c4_of4.log
timeout -k 10 300 python3 tools/bench3d.py --size 512 --dtype f32 --rank-of 8 --steps 40 > $O/c4_of8.log 2>&1 || { echo C48_FAILED; tail -20 $O/c4_of8.log; exit 1; }
tail -1 $O/c4_of8.log
timeout -k 10 400 python3 tools/bench3d.py --size 1024 --dtype f64 --rank-of 8 --steps 16 > $O/c5_of8.log 2>&1 || { echo C5_FAILED; tail -20 $O/c5_of8.log; exit 2; }
tail -1 $O/c5_of8.log
