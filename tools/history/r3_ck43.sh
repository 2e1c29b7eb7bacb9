#!/bin/bash
# round 3 checkpoint 43: step 0's x rows loaded with the prologue's rows (PCS_NM_XEARLY=1): march / slab
# parity, then C3 and c3_cen A/B against loading them after the prologue's PV
set -o pipefail
mkdir -p gpurun_out/r3_ck43
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_march.py tests/test_gpu_slab.py \
  > gpurun_out/r3_ck43/tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck43/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck43/tests.txt
PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py early=pycsou_amd/lib/libpycsou_hip.so \
  late=pycsou_amd/lib/var/xe0/libpycsou_hip.so > gpurun_out/r3_ck43/xe_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck43/xe_ab.txt; exit 1; }
cat gpurun_out/r3_ck43/xe_ab.txt
PCS_KIND=centered PCS_REPS=2 timeout -k 10 400 python -u tools/march_ablate.py early=pycsou_amd/lib/libpycsou_hip.so \
  late=pycsou_amd/lib/var/xe0/libpycsou_hip.so > gpurun_out/r3_ck43/xe_cen_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck43/xe_cen_ab.txt; exit 1; }
cat gpurun_out/r3_ck43/xe_cen_ab.txt
