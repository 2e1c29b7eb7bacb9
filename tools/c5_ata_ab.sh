#!/bin/bash
# C5 (1024^3 fp64): three-pass in-plane chain (PCS_3D_ATA=0, the fp64 default) against the one-launch normal
# operator k_sep2d_nrm<double> (PCS_3D_ATA=1), alternating.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for r in 1 2; do
  for a in 0 1; do
    PCS_3D_ATA=$a timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 2>&1 | tail -1 | sed "s/^/ata$a rep$r /" >> $out/c5_ata_ab.txt || exit 1
  done
done
cat $out/c5_ata_ab.txt
