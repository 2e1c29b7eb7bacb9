#!/bin/bash
# C4 (512^3 fp32, forward K) and C4-centred through tools/bench3d.py for library variants, alternating.
# $1: out dir, $2..: variant names under pycsou_amd/lib/var ("default" = in-tree)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    for k in forward centered; do
      PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --kind $k --steps 40 --warmup 5 2>&1 | tail -1 | sed "s/^/$v $k rep$r /" >> $out/c4_ab.txt || exit 1
    done
  done
done
cat $out/c4_ab.txt
