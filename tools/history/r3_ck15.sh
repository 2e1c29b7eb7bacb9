#!/bin/bash
# round 3 checkpoint 15: general normal-operator march ablations (c3_cen step time)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default nmg1 nmg2 nmg3 prev default; do
  if [ $lib = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$lib/libpycsou_hip.so; fi
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --legs c3_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck15_$lib.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck15_$lib.json').read().splitlines()[-1]); c=d['c3_cen']
print('$lib', 'C3', d['value'], d['roofline']['kernel_ms'], 'c3_cen', c.get('it_per_s'), c.get('kernels_ms'))"
done
