#!/bin/bash
# round 6: does the 12 x 256 fp32 general-K tile win by its row segments or by its plane segmentation?  C4 centred
# at forced segment counts (PCS_3D_NSEG) for the in-tree 12 x 256 tiles and the old 16 x 128 tiles (var g16x128),
# and the forward (folded) kernel at 1 / 2 / 4 / 8 segments
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_nseg
mkdir -p $out
run() {  # label lib nseg kind
  if [ "$2" = default ]; then L=""; else L=pycsou_amd/lib/var/$2/libpycsou_hip.so; fi
  PCS_LIB_PATH=$L PCS_3D_NSEG=$3 timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind $4 2>&1 | tail -1 | sed 's/"workload": "[^"]*", //' | sed "s/^/$1 nseg=$3 /" >> $out/ab.txt
}
for r in 1 2; do
  for n in 0 3 8 14; do run w256r12 default $n centered || exit 1; done
  for n in 2 4 8 16; do run g16x128 g16x128 $n centered || exit 1; done
  for n in 0 2 4 8; do run fold default $n forward || exit 1; done
done
cat $out/ab.txt
