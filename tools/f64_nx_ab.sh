#!/bin/bash
# fp64 C3 legs: env settings A/B (each argument VAR=VALUE or "default"), alternating.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 200 python bench.py --steps 200 --warmup 20 --legs c3_f64,c3_cen_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('$v rep $r', {k: (d[k]['it_per_s'], d[k]['kernels_ms']) for k in ('c3_f64','c3_cen_f64')})" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
