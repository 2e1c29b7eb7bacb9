#!/bin/bash
# C3 headline kernel (k_pds2d_nmarch) workgroups: PCS_NMARCH_SLOTS (0 = default, 3 / CU resident), alternating.
# $1: out dir, $2..: slots
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for r in 1 2; do
  for sl in "$@"; do
    PCS_NMARCH_SLOTS=$sl timeout -k 10 200 python bench.py --steps 400 --warmup 40 --legs "" --volumes "" --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('NMARCH_SLOTS=$sl rep $r', d['value'], d['ms_per_step'])" >> $out/ab.txt || exit 1
  done
done
cat $out/ab.txt
