#!/bin/bash
# C5 (1024^3 fp64, forward K) through tools/bench3d.py for library variants, alternating.  $1: out dir,
# $2..: variant names under pycsou_amd/lib/var ("default" = in-tree)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/c5_ab.txt || exit 1
  done
done
cat $out/c5_ab.txt
