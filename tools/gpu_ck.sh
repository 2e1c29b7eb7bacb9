#!/bin/bash
# Round-4 checkpoint on the GPU box: targeted tests first ($2: pytest selection), then the full
# checkpoint (tools/ck_run.sh: all GPU tests, smoke, bench line, rocprofv3 kernel stats) under gpurun_out/$1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
if [ -n "$2" ]; then
  timeout -k 10 500 python -u -m pytest $2 -x -q --timeout 240 --timeout-method thread > gpurun_out/$1/new_tests.txt 2>&1 \
    || { echo NEW_TESTS_FAILED; tail -40 gpurun_out/$1/new_tests.txt; exit 1; }
  tail -3 gpurun_out/$1/new_tests.txt
fi
[ "$3" = "quick" ] && exit 0
bash tools/ck_run.sh $1
