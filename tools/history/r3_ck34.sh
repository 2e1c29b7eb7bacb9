#!/bin/bash
# round 3 checkpoint 34: cooperative 65th column in the C3 kernel: march parity, A/B against the
# serial branch (PCS_NM_COOP65=0), then the full checkpoint (GPU tests, smoke, bench, kernel stats)
set -o pipefail
mkdir -p gpurun_out/r3_ck34
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_march.py \
  > gpurun_out/r3_ck34/march_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck34/march_tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck34/march_tests.txt
PCS_REPS=4 timeout -k 10 400 python -u tools/march_ablate.py coop=pycsou_amd/lib/libpycsou_hip.so \
  serial=pycsou_amd/lib/var/c65off/libpycsou_hip.so > gpurun_out/r3_ck34/coop65_ab.txt 2>&1 || { tail -20 gpurun_out/r3_ck34/coop65_ab.txt; exit 1; }
cat gpurun_out/r3_ck34/coop65_ab.txt
bash tools/ck_run.sh r3_ck34
