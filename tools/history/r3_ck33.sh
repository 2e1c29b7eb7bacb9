#!/bin/bash
# round 3 checkpoint 33: folded axis-0 pass as the fp32 default: every 3-D GPU test, C4 leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pds.py tests/test_gpu_slab.py -k "3d or folded" \
  > gpurun_out/r3_ck33_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck33_tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck33_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline > gpurun_out/r3_ck33_c4.json 2>gpurun_out/r3_ck33_c4.err || { tail -20 gpurun_out/r3_ck33_c4.err; exit 1; }
tail -c 1500 gpurun_out/r3_ck33_c4.json
