#!/bin/bash
# round 3 checkpoint 17: stencil march at 4 workgroups / CU (128-VGPR budget, tools/build_var.sh smw4 -DPCS_SM_WPE=4)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default smw4 default smw4; do
  if [ $v = default ]; then unset PCS_LIB_PATH PCS_SM_SLOTS; else export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so PCS_SM_SLOTS=1024; fi
  timeout -k 10 300 python bench.py --steps 500 --warmup 50 --legs c2_lap,c2_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck17_$v.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck17_$v.json').read().splitlines()[-1])
print('$v', 'lap', d['c2_lap']['it_per_s'], d['c2_lap']['roofline']['kernel_ms'], 'cen', d['c2_cen']['it_per_s'], d['c2_cen']['roofline']['kernel_ms'])"
done
