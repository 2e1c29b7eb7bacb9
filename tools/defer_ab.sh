#!/bin/bash
# Library variants on the 2-D legs: C3 headline + c2 / c2_lap / c2_cen / c3_cen, alternating.  $1: out dir, $2..: variants
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 400 --warmup 40 --legs c2,c2_lap,c2_cen,c3_cen --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('$v rep $r', 'C3', d['value'], {k: d[k]['it_per_s'] for k in ('c2','c2_lap','c2_cen','c3_cen')})" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
