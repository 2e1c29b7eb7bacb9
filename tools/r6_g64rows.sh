#!/bin/bash
# round 6: k_pds3d_gen<double> tile rows 8 (default) vs 10 / 12 (tools/build_var.sh g64r10|g64r12 -DPCS_3DG_ROWS64=..)
# parity of the 12-row variant on the 3-D general-K tests, then C5 centred through bench3d.py, alternating
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g64rows
mkdir -p $out
PCS_LIB_PATH=pycsou_amd/lib/var/g64r12/libpycsou_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 250 \
  --timeout-method thread tests/test_gpu_pds.py -k "general_k or ragged or 128_fp64" tests/test_gpu_slab.py::test_slab3d_general_k_bitwise \
  > $out/tests_r12.txt 2>&1 || { tail -20 $out/tests_r12.txt; exit 1; }
tail -2 $out/tests_r12.txt
for r in 1 2; do
  for v in default g64r12 g64r10; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 --kind centered 2>&1 | tail -1 | sed "s/^/$v rep$r /" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
