#!/bin/bash
# round 3 checkpoint 12: 16-row fp32 tiles in k_pds3d_gen -- parity (3-D general K + slabs) and C4 centred timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pds.py tests/test_gpu_slab.py -k "pds3d or slab3d" > gpurun_out/r3_ck12_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3_ck12_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in centered forward centered; do
  timeout -k 10 200 python tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4 --kind $k 2>/dev/null | tail -1 || exit $?
done
timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 6 --warmup 2 --kind centered 2>/dev/null | tail -1 || exit $?
