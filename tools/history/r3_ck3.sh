#!/bin/bash
# round 3 checkpoint 3: FFT Convolve2D parity + Lanczos, conv63 / c3_cen legs, PMC of the stencil march
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fftconv.py "tests/test_gpu_ops.py::test_lipschitz_lanczos" "tests/test_gpu_ops.py::test_lipschitz_scalable" > gpurun_out/r3_ck3_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_ck3_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --legs conv63,c3_cen --volumes "" --no-cpu-baseline > gpurun_out/r3_ck3_bench.json 2> gpurun_out/r3_ck3_bench.err || exit $?
PCS_PROBLEM=c2_lap bash tools/prof_nm.sh r3_prof_lap k_pds2d_smarch || exit $?
PCS_PROBLEM=c2_cen bash tools/prof_nm.sh r3_prof_cen k_pds2d_smarch || exit $?
