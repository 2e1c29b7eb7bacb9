#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-slabg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_slab.py -k "graph or native_loop" -x -v --timeout 200 --timeout-method thread > $O/t.txt 2>&1 || { echo T_FAILED; tail -40 $O/t.txt; exit 1; }
tail -2 $O/t.txt
timeout -k 10 300 python3 tools/slab_graph_probe.py > $O/probe.txt 2>&1 || { echo P_FAILED; tail -20 $O/probe.txt; exit 2; }
cat $O/probe.txt
