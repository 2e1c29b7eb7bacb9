#!/bin/bash
# round 6: C5 rank-share link model (one rank of 8, forward and centred K) after the 12-row fp64 tiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_share2; mkdir -p $O
timeout -k 10 300 python -u tools/bench3d.py --size 1024 --dtype f64 --rank-of 8 --steps 16 --one-gpu-ms 23.0 > $O/share_c5.txt 2>&1 || { echo "share c5 failed"; tail $O/share_c5.txt; exit 1; }
tail -1 $O/share_c5.txt
timeout -k 10 300 python -u tools/bench3d.py --size 1024 --dtype f64 --rank-of 8 --steps 16 --kind centered --one-gpu-ms 24.8 > $O/share_c5cen.txt 2>&1 || { echo "share c5cen failed"; tail $O/share_c5cen.txt; exit 1; }
tail -1 $O/share_c5cen.txt
