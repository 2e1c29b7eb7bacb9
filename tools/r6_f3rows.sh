#!/bin/bash
# round 6: k_pds3d<double> (forward K) tile rows 8 (in-tree) vs 12 (var f3r12, -DPCS_3D_ROWS64=12): 3-D tests of the
# variant, then C5 forward through bench3d.py, alternating
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_f3rows
mkdir -p $out
PCS_LIB_PATH=pycsou_amd/lib/var/f3r12/libpycsou_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_pds.py -k "3d" tests/test_gpu_slab.py -k "3d or slab3d" tests/test_gpu_fullsize.py > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2; do
  for v in default f3r12; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
