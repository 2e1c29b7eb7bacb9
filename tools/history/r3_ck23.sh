#!/bin/bash
# round 3 checkpoint 23: grid-size sweep of the stencil march at 2048^2 (PCS_SM_SLOTS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for sl in 768 512 640 1024 1280 768; do
  PCS_SM_SLOTS=$sl timeout -k 10 200 python bench.py --steps 500 --warmup 50 --legs c2_lap,c2_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck23_$sl.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck23_$sl.json').read().splitlines()[-1])
print('$sl', 'lap', d['c2_lap']['it_per_s'], d['c2_lap']['roofline']['kernel_ms'], 'cen', d['c2_cen']['it_per_s'], d['c2_cen']['roofline']['kernel_ms'])"
done
