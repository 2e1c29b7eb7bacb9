#!/bin/bash
# k_sep2d_nrm library variants on the C4 volume (fp32) and C5 volume (fp64), alternating.  $1: out dir,
# $2..: variant names under pycsou_amd/lib/var ("default" = in-tree)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L PCS_ATA_KERNELS=2pass PCS_ATA_CASES=512:512:f32,1024:1024:f64,1:4096:f64 timeout -k 10 200 python tools/ata_probe.py \
      | sed "s/^/rep$r $v /" >> $out/nrm_var_ab.txt || exit 1
  done
done
cat $out/nrm_var_ab.txt
