#!/bin/bash
# Round 6: the deep-halo 2-D slab loop tests, then the whole slab suite
set -o pipefail
O=gpurun_out/r6_4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slab.py -k deep \
  > $O/deep.txt 2>&1 || { echo "deep tests failed"; grep -E "^E |FAILED|Error" $O/deep.txt | head -30; exit 1; }
tail -3 $O/deep.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_slab.py \
  > $O/slab.txt 2>&1 || { echo "slab tests failed"; grep -E "^E |FAILED" $O/slab.txt | head -30; exit 1; }
tail -3 $O/slab.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_bench_launch.py \
  > $O/launch.txt 2>&1 || { echo "launch tests failed"; grep -E "^E |FAILED" $O/launch.txt | head -30; tail -20 $O/launch.txt; exit 1; }
tail -3 $O/launch.txt
