#!/bin/bash
# round 3 checkpoint 24: cost of the GEN march's merged extra-column branch (nmg1: -DPCS_NMG_ABL=1, timing only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default nmg1 default nmg1; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs c3_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck24_$v.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck24_$v.json').read().splitlines()[-1]); c=d['c3_cen']
print('$v', 'c3_cen', c.get('it_per_s'), c.get('kernels_ms'))"
done
