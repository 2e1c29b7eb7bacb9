#!/bin/bash
# round 3 checkpoint 13: fused normal-operator march for backward / centred K -- parity, slabs,
# C3 forward A/B against the previous library, c3_cen timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_smarch.py tests/test_gpu_slab.py tests/test_gpu_march.py > gpurun_out/r3_ck13_tests.txt 2>&1
rc=$?
tail -15 gpurun_out/r3_ck13_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in new prev new prev; do
  if [ $lib = prev ]; then export PCS_LIB_PATH=pycsou_amd/lib/var/prev/libpycsou_hip.so; else unset PCS_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs c3_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck13_$lib.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck13_$lib.json').read().splitlines()[-1]); c=d['c3_cen']
print('$lib', 'C3', d['value'], d['roofline']['kernel_ms'], 'c3_cen', c.get('it_per_s'), c.get('kernels_ms'))"
done
