#!/bin/bash
# round 3 checkpoint 21: b loads a step ahead in the normal-operator march (tools/build_var.sh bah -DPCS_NM_BAHEAD=1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default bah default bah default bah; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs c3_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck21_$v.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck21_$v.json').read().splitlines()[-1]); c=d['c3_cen']
print('$v', 'C3', d['value'], d['roofline']['kernel_ms'], 'c3_cen', c.get('it_per_s'), c.get('kernels_ms'))"
done
