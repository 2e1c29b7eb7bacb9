#!/bin/bash
# Round 6 checkpoint: the whole GPU suite and smoke(), then the default bench line
set -o pipefail
O=gpurun_out/${R6_OUT:-r6_full}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -5 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
