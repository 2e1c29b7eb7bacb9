#!/bin/bash
# round 3 checkpoint 25: cooperative extra columns in the GEN normal-operator march -- parity + c3_cen timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_smarch.py tests/test_gpu_slab.py -k "smarch or fused or sep_cen or general_k" > gpurun_out/r3_ck25_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3_ck25_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs c3_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck25_$i.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck25_$i.json').read().splitlines()[-1]); c=d['c3_cen']
print('coop', 'C3', d['roofline']['kernel_ms'], 'c3_cen', c.get('it_per_s'), c.get('kernels_ms'))"
done
