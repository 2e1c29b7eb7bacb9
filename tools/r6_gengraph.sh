#!/bin/bash
# round 6: generic PDS loop as hipGraph chunks -- parity tests (graph vs eager, reference goldens of the solver
# subclasses and stacks), then tools/bench_generic.py with and without the graphs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_gengraph; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic_graph.py \
  tests/test_gpu_solvers.py tests/test_gpu_stacks.py > $O/tests.txt 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.txt | head -30; tail -5 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python -u tools/bench_generic.py > $O/bench_graph.txt 2>&1 || { tail -5 $O/bench_graph.txt; exit 1; }
PCS_GENERIC_GRAPH=0 timeout -k 10 200 python -u tools/bench_generic.py > $O/bench_eager.txt 2>&1 || { tail -5 $O/bench_eager.txt; exit 1; }
cat $O/bench_graph.txt $O/bench_eager.txt
timeout -k 10 200 python -u tools/bench_generic.py 256 > $O/bench_graph256.txt 2>&1 || { tail -5 $O/bench_graph256.txt; exit 1; }
PCS_GENERIC_GRAPH=0 timeout -k 10 200 python -u tools/bench_generic.py 256 > $O/bench_eager256.txt 2>&1 || { tail -5 $O/bench_eager256.txt; exit 1; }
grep problem $O/bench_graph256.txt $O/bench_eager256.txt
