#!/bin/bash
# fp64 C3 legs with grad F = N x - Conv^T y formed by the normal-operator kernel (default) against N x alone +
# the subtraction in the step (PCS_NX_SUB=0), alternating.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for r in 1 2; do
  for v in 1 0; do
    PCS_NX_SUB=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --legs c3_f64,c3_cen_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('nx_sub=$v rep $r', {k: (d[k]['it_per_s'], d[k]['kernels_ms'], d[k]['roofline']['frac']) for k in ('c3_f64','c3_cen_f64')})" >> $out/nxsub_ab.txt || exit 1
  done
done
cat $out/nxsub_ab.txt
