#!/bin/bash
# c3_nonsep with PCS_CORR_ROUNDS = 1 / 2 / 3 (rounds of the resident correlation workgroups), alternating.  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    PCS_CORR_ROUNDS=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --legs c3_nonsep --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('rounds=$v rep $r', d['c3_nonsep']['it_per_s'], d['c3_nonsep']['kernels_ms'])" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
