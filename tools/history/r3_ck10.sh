#!/bin/bash
# round 3 checkpoint 10: 3-D backward / centred K (k_pds3d_gen) parity + slabs, generic-path leg,
# c4_cen volume leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_pds.py -k "pds3d" tests/test_gpu_slab.py -k "slab3d or pds3d" > gpurun_out/r3_ck10_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_ck10_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --legs cps_inpaint --volumes "c4:512:f32:20,c4_cen:512:f32:20:centered" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck10_bench.json 2> gpurun_out/r3_ck10_bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck10_bench.json').read().splitlines()[-1])
for k in ('cps_inpaint','volume_c4','volume_c4_cen'): print(k, d.get(k))"
