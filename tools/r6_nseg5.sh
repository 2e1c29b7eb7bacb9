#!/bin/bash
# round 6: C5 (1024^3 fp64) update kernels at forced plane-segment counts (PCS_3D_NSEG; 0 = the makespan model: 7)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_nseg5; mkdir -p $O
for kind in forward centered; do
  for n in 0 4 11 14 21; do
    PCS_3D_NSEG=$n timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 --kind $kind 2>&1 | tail -1 | sed 's/"workload": "[^"]*", //' | sed "s/^/$kind nseg=$n /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
