#!/bin/bash
# round 6: k_pds3d_gen column-border tiles on their own code form (row axis interior; in-tree) against the
# all-edge-rules form (var g3nrf: -DPCS_3DG_ROWFORM=0): 3-D tests of the in-tree build, then C4 centred and C5 centred
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g3rowform
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_pds.py -k "3d" tests/test_gpu_slab.py -k "3d or slab3d" tests/test_gpu_fullsize.py > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2 3; do
  for v in default g3nrf; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind centered 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
for v in default g3nrf; do
  if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 --kind centered 2>&1 | tail -1 | sed "s/^/$v c5cen /" >> $out/ab.txt || exit 1
done
cat $out/ab.txt
