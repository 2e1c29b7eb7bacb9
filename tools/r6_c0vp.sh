#!/bin/bash
# round 6: the fp32 axis-0 pass (k_conv0_rta) with 2 voxels per thread (in-tree) vs 1 (var c0vp1): 3-D tests of the
# in-tree build (the folded kernel stays bitwise this pass), then C4 centred alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_c0vp; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_pds.py tests/test_gpu_slab.py \
  tests/test_gpu_ops.py -k "3d or conv0 or axis0 or volume or conv1d" > $O/tests.txt 2>&1 || { grep -E "^E |FAILED" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in default c0vp1; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind centered 2>&1 | tail -1 | sed 's/"workload": "[^"]*", //' | sed "s/^/$v rep$r /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
