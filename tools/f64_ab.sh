#!/bin/bash
# fp64 C3 legs, A/B of library variants (alternating reps): $1 out dir, $2.. variant names under
# pycsou_amd/lib/var ("default" = the in-tree library)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --legs c3_f64,c3_cen_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('$v rep $r', {k: (d[k]['it_per_s'], d[k]['kernels_ms']) for k in ('c3_f64','c3_cen_f64')})" >> $out/f64_ab.txt || exit 1
  done
done
