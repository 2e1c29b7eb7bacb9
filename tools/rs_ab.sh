#!/bin/bash
# 32-row steps (PCS_SM_RS=2) of the general-stencil march: parity of every fp32 K at RS = 2, then the
# 2048^2 / 4096^2 Laplacian / centred probes at RS = 1 and 2 (alternating reps).  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
PCS_SM_RS=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_smarch.py -x -q --timeout 200 > $out/tests_rs2.txt 2>&1 \
  || { tail -30 $out/tests_rs2.txt; exit 1; }
tail -2 $out/tests_rs2.txt
for r in 1 2; do
  for rs in 1 2; do
    PCS_SM_RS=$rs timeout -k 10 200 python tools/sm_probe.py | sed "s/^/n2048 rs$rs rep$r /" >> $out/rs_ab.txt || exit 1
  done
done
for rs in 1 2; do
  PCS_N=4096 PCS_SM_RS=$rs timeout -k 10 200 python tools/sm_probe.py | sed "s/^/n4096 rs$rs /" >> $out/rs_ab.txt || exit 1
done
cat $out/rs_ab.txt
