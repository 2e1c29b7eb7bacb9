#!/bin/bash
# round 3 checkpoint 36: GEN (centred-K C3) extra columns reduced by DPP instead of ds_bpermute shuffles:
# nmarch parity, A/B on c3_cen (PCS_KIND=centered)
set -o pipefail
mkdir -p gpurun_out/r3_ck36
export TMPDIR=/tmp
true \
  > gpurun_out/r3_ck36/tests.txt 2>&1 || { tail -40 gpurun_out/r3_ck36/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck36/tests.txt
PCS_KIND=centered PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py dpp=pycsou_amd/lib/libpycsou_hip.so \
  shfl=pycsou_amd/lib/var/dpp0/libpycsou_hip.so > gpurun_out/r3_ck36/dpp_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck36/dpp_ab.txt; exit 1; }
cat gpurun_out/r3_ck36/dpp_ab.txt
