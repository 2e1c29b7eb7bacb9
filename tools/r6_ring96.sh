#!/bin/bash
# round 6: folded 3-D kernel's ring loads as one 12-B access (in-tree) vs three 4-B ones (var r96off): 3-D tests of the
# in-tree build (the fold stays bitwise the separate axis-0 pass), then C4 forward alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_ring96; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_pds.py tests/test_gpu_slab.py \
  tests/test_gpu_long2.py -k "3d" > $O/tests.txt 2>&1 || { grep -E "^E |FAILED" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in default r96off; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 2>&1 | tail -1 | sed 's/"workload": "[^"]*", //' | sed "s/^/$v rep$r /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
