#!/bin/bash
# k_sep2d_nrm grid sweep (PCS_ATA_SLOTS): C4 volume fp32, C3 plane fp64, C5 volume fp64.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for sl in 256 384 512 640 768; do
  PCS_ATA_KERNELS=2pass PCS_ATA_CASES=512:512:f32 PCS_ATA_SLOTS=$sl timeout -k 10 120 python tools/ata_probe.py | sed "s/^/slots$sl /" >> $out/nrm_slots.txt || exit 1
done
for sl in 256 512 768 1024 1536 2048; do
  PCS_ATA_KERNELS=2pass PCS_ATA_CASES=1:4096:f64 PCS_ATA_SLOTS=$sl timeout -k 10 120 python tools/ata_probe.py | sed "s/^/slots$sl /" >> $out/nrm_slots.txt || exit 1
done
for sl in 512 1024 1536 2048; do
  PCS_ATA_KERNELS=2pass PCS_ATA_CASES=1024:1024:f64 PCS_ATA_SLOTS=$sl timeout -k 10 120 python tools/ata_probe.py | sed "s/^/slots$sl /" >> $out/nrm_slots.txt || exit 1
done
cat $out/nrm_slots.txt
