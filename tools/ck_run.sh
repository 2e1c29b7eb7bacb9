#!/bin/bash
# Checkpoint: GPU tests, bench line, kernel-trace stats of the bench (dir under gpurun_out/ = $1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${1:-ck}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${1:-ck}/gpu_tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${1:-ck}/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${1:-ck}/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${1:-ck}/smoke.txt 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/${1:-ck}/smoke.txt; exit 4; }
tail -1 gpurun_out/${1:-ck}/smoke.txt
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/${1:-ck}/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${1:-ck}/bench.log; exit 2; }
tail -1 gpurun_out/${1:-ck}/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${1:-ck}/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${1:-ck}/prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/${1:-ck}/prof.log; exit 3; }
# the per-dispatch trace is tens of MB (gpurun_out/ comes back only under 64 MiB): keep the stats
find gpurun_out/${1:-ck}/prof \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
echo ALL_OK
