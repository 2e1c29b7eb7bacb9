#!/bin/bash
# C4 centred K (k_pds3d_gen): plane-segment task target (PCS_3D_TARGET; 0 = default one task per CU), alternating
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for t in "$@"; do
    PCS_3D_TARGET=$t timeout -k 10 200 python tools/bench3d.py --size 512 --dtype f32 --kind centered --steps 20 --warmup 4 2>&1 | tail -1 | sed "s/^/C4cen target$t rep$r /" >> $out/sweep.txt || exit 1
  done
done
cat $out/sweep.txt
