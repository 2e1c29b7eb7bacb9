#!/bin/bash
# A/B of the fp32 correlation kernels (PCS_CORR_PK=1 packed two-row kernel vs 0 scalar), 4096^2, k = 7/15/31,
# alternating 3 reps, then the c3_nonsep bench leg with each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
for r in 1 2 3; do
  for pk in 1 0; do
    echo "PK=$pk rep $r" >> gpurun_out/$1/corr_ab.txt
    PCS_CORR_PK=$pk timeout -k 10 120 python tools/conv2d_bench.py --ks 7,15,31 --dtypes f32 >> gpurun_out/$1/corr_ab.txt 2>&1 || exit 1
  done
done
for pk in 1 0; do
  PCS_CORR_PK=$pk timeout -k 10 300 python bench.py --steps 200 --warmup 20 --legs c3_nonsep --volumes "" --no-cpu-baseline > gpurun_out/$1/nonsep_pk$pk.json 2>&1 || exit 1
done
