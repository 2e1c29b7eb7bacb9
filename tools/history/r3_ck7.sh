#!/bin/bash
# round 3 checkpoint 7: slab generality after the fixes + stencil/FFT parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_smarch.py tests/test_gpu_fftconv.py tests/test_gpu_march.py > gpurun_out/r3_ck7_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_ck7_tests.txt
exit $rc
