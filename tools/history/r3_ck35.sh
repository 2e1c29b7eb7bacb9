#!/bin/bash
# round 3 checkpoint 35: C3 kernel PV / update / P6 in the column layout (PCS_NM_COLS=1): march and slab
# parity, then A/B against the row layout (PCS_NM_COLS=0)
set -o pipefail
mkdir -p gpurun_out/r3_ck35
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_march.py tests/test_gpu_slab.py \
  > gpurun_out/r3_ck35/tests.txt 2>&1 || { tail -40 gpurun_out/r3_ck35/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck35/tests.txt
PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py cols=pycsou_amd/lib/libpycsou_hip.so \
  rows=pycsou_amd/lib/var/cols0/libpycsou_hip.so > gpurun_out/r3_ck35/cols_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck35/cols_ab.txt; exit 1; }
cat gpurun_out/r3_ck35/cols_ab.txt
