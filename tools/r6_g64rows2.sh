#!/bin/bash
# round 6: fp64 general-K update at 12 rows with the makespan-balanced segment count (in-tree) against 12 rows
# with one segment (var g64r12) and 8 rows (var g64r8); 3-D tests of the in-tree build first
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g64rows2
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_pds.py -k "3d" \
  tests/test_gpu_slab.py -k "3d or slab3d" tests/test_gpu_fullsize.py > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2; do
  for v in default g64r12 g64r8; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 --kind centered 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
