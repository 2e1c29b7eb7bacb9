#!/bin/bash
# round 6: k_pds3d_gen<float> 16 x 128 tiles (in-tree) against 256-column tiles (1 KB row segments) with 1024-thread
# workgroups and one prefetch set: w256r12 (12 rows), w256r8 (8 rows).  3-D tests of w256r12, then C4 centred
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g32w
mkdir -p $out
PCS_LIB_PATH=pycsou_amd/lib/var/w256r12/libpycsou_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_pds.py -k "3d" tests/test_gpu_slab.py -k "3d or slab3d" > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2; do
  for v in default w256r12 w256r8; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind centered 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
