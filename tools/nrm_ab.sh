#!/bin/bash
# k_sep2d_nrm variants (tools/ata_probe.py: 512^3 fp32, 1024^3 fp64), alternating reps, then a grid sweep
# of the default build.  $1: out dir, $2..: variant names under pycsou_amd/lib/var ("default" = in-tree)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 200 python tools/ata_probe.py 2>&1 | grep 2pass | sed "s/^/rep$r /" >> $out/nrm_ab.txt || exit 1
  done
done
for sl in 512 1024; do
  PCS_ATA_SLOTS=$sl timeout -k 10 200 python tools/ata_probe.py 2>&1 | grep 2pass | sed "s/^/slots$sl /" >> $out/nrm_ab.txt || exit 1
done
cat $out/nrm_ab.txt
