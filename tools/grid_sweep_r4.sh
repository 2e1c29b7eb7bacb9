#!/bin/bash
# Grid sweeps on the final kernels: the 3-D update's task count (PCS_3D_TARGET: C4 / C5) and the fp64 2-D march
# step's workgroups (PCS_SM_SLOTS: c3_f64).  $1: out dir
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for t in 0 512 1024 2048; do
  PCS_3D_TARGET=$t timeout -k 10 200 python tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4 2>&1 | tail -1 | sed "s/^/C4 target$t /" >> $out/sweep.txt || exit 1
done
for t in 0 2048 4096 8192; do
  PCS_3D_TARGET=$t timeout -k 10 300 python tools/bench3d.py --size 1024 --dtype f64 --steps 8 --warmup 2 2>&1 | tail -1 | sed "s/^/C5 target$t /" >> $out/sweep.txt || exit 1
done
for sl in 0 256 1024 1536; do
  PCS_SM_SLOTS=$sl timeout -k 10 200 python bench.py --steps 100 --warmup 10 --legs c3_f64 --volumes "" --no-cpu-baseline 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('c3_f64 SM_SLOTS=$sl', d['c3_f64']['it_per_s'], d['c3_f64']['kernels_ms'])" >> $out/sweep.txt || exit 1
done
cat $out/sweep.txt
