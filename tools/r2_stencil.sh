#!/bin/bash
# round-2: general-stencil fused PDS step parity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-stencil}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py -x -v --timeout 120 --timeout-method thread > $O/t_stencil.txt 2>&1 || { echo STENCIL_FAILED; tail -60 $O/t_stencil.txt; exit 1; }
tail -3 $O/t_stencil.txt
