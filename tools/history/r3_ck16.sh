#!/bin/bash
# round 3 checkpoint 16: cost of the forward kernel's 65th-column branch (C3 step time)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default nmf4 default nmf4; do  # nmf4: tools/build_var.sh nmf4 -DPCS_NMG_ABL=4
  if [ $lib = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$lib/libpycsou_hip.so; fi
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs "" --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck16_$lib.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck16_$lib.json').read().splitlines()[-1])
print('$lib', 'C3', d['value'], d['roofline']['kernel_ms'])"
done
