#!/bin/bash
# round 3 checkpoint 41: C5 (1024^3 fp64) with the in-plane normal operator (PCS_3D_ATA=1: k_sep2d_nrm,
# 15 words / voxel) against the three-pass chain (0: 17 words), alternating
set -o pipefail
mkdir -p gpurun_out/r3_ck41
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 1 0; do
    PCS_3D_ATA=$v timeout -k 10 300 python bench.py --steps 10 --warmup 4 --legs "" --volumes c5:1024:f64:10 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck41/ata$v$rep.json 2>gpurun_out/r3_ck41/ata$v$rep.err || { tail -20 gpurun_out/r3_ck41/ata$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck41/ata$v$rep.json').read().splitlines()[-1]); c=d['volume_c5']
print('ata $v rep $rep', c['it_per_s'], c['ms_per_iter'])" | tee -a gpurun_out/r3_ck41/ab.txt
  done
done
