#!/bin/bash
# round 3: general-stencil march kernel -- parity tests, then the 2-D stencil bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_smarch.py tests/test_gpu_stencil.py > gpurun_out/r3_sm_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_sm_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 300 --warmup 30 --legs c2,c2_lap,c2_cen --volumes "" --no-cpu-baseline > gpurun_out/r3_sm_bench.json 2> gpurun_out/r3_sm_bench.err
