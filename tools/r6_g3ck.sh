#!/bin/bash
# round 6: 3-D GPU tests (incl. full-size C4 / C5) of the in-tree build, then C4 centred / C5 centred bench3d lines
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_g3ck
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_pds.py tests/test_gpu_slab.py tests/test_gpu_fullsize.py tests/test_gpu_long2.py tests/test_gpu_determinism.py -k "3d or c5 or c4" > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 300 python tools/bench3d.py --size 512 --dtype f32 --steps 40 --warmup 6 --kind centered 2>&1 | tail -1 | sed "s/^/c4cen /" >> $out/ab.txt || exit 1
timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 10 --warmup 3 --kind centered 2>&1 | tail -1 | sed "s/^/c5cen /" >> $out/ab.txt || exit 1
cat $out/ab.txt
