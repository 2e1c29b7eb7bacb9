#!/bin/bash
# round 6: k_pds3d_gen<float> 512-thread workgroups with two prefetch register sets (in-tree) against 1024-thread
# workgroups with one set (var g32n1k: -DPCS_3DG_NT32=1024 -DPCS_3DG_SETS32=1, 4 waves / SIMD, no spills): 3-D tests
# of the variant, then C4 centred through bench3d.py, alternating
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g32nt
mkdir -p $out
PCS_LIB_PATH=pycsou_amd/lib/var/g32n1k/libpycsou_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_pds.py -k "3d" tests/test_gpu_slab.py -k "3d or slab3d" > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2 3; do
  for v in default g32n1k; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind centered 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
