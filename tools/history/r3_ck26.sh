#!/bin/bash
# round 3 checkpoint 26: N-D (ndim > 3) derivatives / Gradient / Convolve1D
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_stacks.py \
  "tests/test_gpu_pds.py::test_pds_4d_gradient_generic_vs_oracle" "tests/test_gpu_pds.py::test_pds3d_general_k_vs_oracle" \
  > gpurun_out/r3_ck26_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_ck26_tests.txt; exit $rc
