#!/bin/bash
# fp64 2-D march step workgroups (PCS_SM_SLOTS: 0 = default), both fp64 C3 legs, alternating.  $1: out dir, $2..: slots
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for sl in "$@"; do
    PCS_SM_SLOTS=$sl timeout -k 10 200 python bench.py --steps 200 --warmup 20 --legs c3_f64,c3_cen_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('SM_SLOTS=$sl rep $r', {k: (d[k]['it_per_s'], d[k]['kernels_ms']) for k in ('c3_f64','c3_cen_f64')})" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
