#!/bin/bash
# fp64 C3 (4096^2) grid sweeps: the march step's workgroups (PCS_SM_SLOTS) and the N x pass's (PCS_ATA_SLOTS)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
for s in 0 256 384 768 1024; do
  PCS_SM_SLOTS=$s timeout -k 10 200 python bench.py --steps 100 --warmup 10 --legs c3_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1])['c3_f64']; print('SM_SLOTS=$s', d['it_per_s'], d['kernels_ms'])" >> gpurun_out/$1/f64_sweep.txt || exit 1
done
for s in 256 512 768 1024; do
  PCS_ATA_SLOTS=$s timeout -k 10 200 python bench.py --steps 100 --warmup 10 --legs c3_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1])['c3_f64']; print('ATA_SLOTS=$s', d['it_per_s'], d['kernels_ms'])" >> gpurun_out/$1/f64_sweep.txt || exit 1
done
