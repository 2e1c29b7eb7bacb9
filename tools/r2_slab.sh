#!/bin/bash
# round-2: multi-GPU transport tests (one GPU: in-process slabs, gloo processes, 1-rank RCCL)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-slab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py -x -v --timeout 300 --timeout-method thread > $O/t_slab.txt 2>&1 || { echo SLAB_FAILED; tail -60 $O/t_slab.txt; exit 1; }
tail -3 $O/t_slab.txt
