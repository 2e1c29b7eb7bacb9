#!/bin/bash
# round 3 checkpoint 38: nt (streaming) cache policy on the march's x / z / b loads (PCS_NM_LAUX=2), A/B on
# C3 and on the centred-K C3
set -o pipefail
mkdir -p gpurun_out/r3_ck38
export TMPDIR=/tmp
PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py dflt=pycsou_amd/lib/libpycsou_hip.so \
  nt=pycsou_amd/lib/var/nt/libpycsou_hip.so > gpurun_out/r3_ck38/nt_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck38/nt_ab.txt; exit 1; }
cat gpurun_out/r3_ck38/nt_ab.txt
PCS_KIND=centered PCS_REPS=2 timeout -k 10 400 python -u tools/march_ablate.py dflt=pycsou_amd/lib/libpycsou_hip.so \
  nt=pycsou_amd/lib/var/nt/libpycsou_hip.so > gpurun_out/r3_ck38/nt_cen_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck38/nt_cen_ab.txt; exit 1; }
cat gpurun_out/r3_ck38/nt_cen_ab.txt
