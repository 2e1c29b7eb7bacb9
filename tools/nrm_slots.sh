#!/bin/bash
# k_sep2d_nrm grids: the default (one task per workgroup) against PCS_NRM_GRIDX=k (k x the resident slots,
# each workgroup a contiguous run of tasks).  C4 volume fp32, C5 volume fp64, C3 plane fp64.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
run() {  # case gridx ("" = default)
  PCS_ATA_KERNELS=2pass PCS_ATA_CASES=$1 PCS_NRM_GRIDX=$2 timeout -k 10 120 python tools/ata_probe.py \
    | sed "s/^/gridx[$2] /" >> $out/nrm_slots.txt
}
for r in 1 2; do
  for c in 512:512:f32 1024:1024:f64 1:4096:f64; do
    for gx in "" 1 8; do run $c "$gx" || exit 1; done
  done
done
cat $out/nrm_slots.txt
