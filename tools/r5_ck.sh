#!/bin/bash
# Round-5 GPU step: targeted tests ($2: pytest selection, may be empty), then optional probes ($3: a
# shell snippet), all under gpurun_out/$1; every GPU step under its own time limit, chained with &&
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -x -q --timeout 240 --timeout-method thread > $out/tests.txt 2>&1 \
    || { echo TESTS_FAILED; tail -40 $out/tests.txt; exit 1; }
  tail -3 $out/tests.txt
fi
if [ -n "$3" ]; then
  bash -o pipefail -c "$3" > $out/probe.txt 2>&1 || { echo PROBE_FAILED; tail -40 $out/probe.txt; exit 2; }
  tail -40 $out/probe.txt
fi
echo STEP_OK
