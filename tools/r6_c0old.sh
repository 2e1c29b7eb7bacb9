#!/bin/bash
# round 6: C5 forward volume leg with the in-tree axis-0 pass (VP template, fp64 at VP = 1) vs the previous kernel
# (var c0old), alternating; bench.py volume legs only
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_c0old; mkdir -p $O
for r in 1 2; do
  for v in default c0old; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --legs "" --volumes c5:1024:f64:10 --no-cpu-baseline > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/run.json')); v=d['volume_c5']
print('$v rep$r', v['it_per_s'], {n: p['kernel_ms'] for n, p in v['roofline']['parts'].items()})
" | tee -a $O/ab.txt
  done
done
