#!/bin/bash
# round 6: GEN march extra columns' PV / update before the own PV items (in-tree) vs after (var xf0, -DPCS_NMG_XFIRST=0)
# GEN tests of the in-tree build, then C3 centred timing alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_xfirst; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_march.py tests/test_gpu_determinism.py \
  tests/test_gpu_fullsize.py tests/test_gpu_long.py tests/test_gpu_slab.py -k "cen or gen or backward or centered or determin or general" > $O/tests.txt 2>&1 || { grep -E "^E |FAILED" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
PCS_KIND=centered timeout -k 10 400 python3 tools/march_ablate.py base=pycsou_amd/lib/libpycsou_hip.so xf0=pycsou_amd/lib/var/xf0/libpycsou_hip.so > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
tail -3 $O/ab.txt
