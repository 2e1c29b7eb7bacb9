#!/bin/bash
# round 3 checkpoint 37: (1) C3 A/B of PV read chunks
# of 4 rows (PCS_NM_PF=4) with the cooperative 65th column, (2) PMC profile of the C3 kernel as built
set -o pipefail
mkdir -p gpurun_out/r3_ck37
export TMPDIR=/tmp
PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py pf2=pycsou_amd/lib/libpycsou_hip.so \
  pf4=pycsou_amd/lib/var/pf4/libpycsou_hip.so > gpurun_out/r3_ck37/pf_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck37/pf_ab.txt; exit 1; }
cat gpurun_out/r3_ck37/pf_ab.txt
bash tools/prof_nm.sh r3_ck37/prof_nm k_pds2d_nmarch && cat gpurun_out/r3_ck37/prof_nm/traffic.json
