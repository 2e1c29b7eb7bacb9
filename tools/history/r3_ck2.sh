#!/bin/bash
# round 3 checkpoint 2: parity of the new paths + stencil legs + a grid sweep of the march step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_smarch.py tests/test_gpu_march.py tests/test_gpu_pds.py tests/test_gpu_slab.py "tests/test_gpu_ops.py::test_lipschitz_lanczos" "tests/test_gpu_ops.py::test_lipschitz_scalable" > gpurun_out/r3_ck2_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_ck2_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 300 --warmup 30 --legs c2_lap,c2_cen,c3_cen --volumes "" --no-cpu-baseline > gpurun_out/r3_ck2_bench.json 2> gpurun_out/r3_ck2_bench.err || exit $?
for sl in 512 1024 1536; do
  PCS_SM_SLOTS=$sl timeout -k 10 200 python bench.py --steps 300 --warmup 30 --legs c2_lap,c2_cen --volumes "" --no-cpu-baseline > gpurun_out/r3_ck2_sweep_$sl.json 2>/dev/null || exit $?
done
