#!/bin/bash
# A/B of k_pds3d_gen tile / occupancy variants on C4 512^3 fp32 with the centred K (tools/bench3d.py),
# alternating 2 reps: default (16-row tiles), g8 (8-row tiles), g8m2 (8-row tiles, 2 workgroups / CU budget);
# then the 3-D general-K parity tests with each variant library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
for r in 1 2; do
  for v in default g8 g8m2; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    echo "$v rep $r: $(PCS_LIB_PATH=$L timeout -k 10 200 python tools/bench3d.py --size 512 --dtype f32 --kind centered --steps 20 --warmup 4 2>/dev/null | tail -1)" >> gpurun_out/$1/g3d_ab.txt || exit 1
  done
done
for v in g8 g8m2; do
  PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so timeout -k 10 300 python -m pytest tests/test_gpu_pds.py tests/test_gpu_slab.py -k "3d" -x -q --timeout 200 > gpurun_out/$1/g3d_tests_$v.txt 2>&1 || { echo "TESTS $v FAILED"; tail -20 gpurun_out/$1/g3d_tests_$v.txt; exit 1; }
  tail -1 gpurun_out/$1/g3d_tests_$v.txt
done
