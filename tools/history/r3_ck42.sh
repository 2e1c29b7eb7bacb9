#!/bin/bash
# round 3 checkpoint 42: fifth-column loads only where kept (pt: group 15; stencil march: groups 0 / 15):
# pds / smarch / slab tests, then 2-D legs A/B against every group loading it (PCS_PT_E5=0 PCS_SM_E5=0),
# then the C5 ATA A/B (tools/r3_ck41.sh)
set -o pipefail
mkdir -p gpurun_out/r3_ck42
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_smarch.py tests/test_gpu_pds.py tests/test_gpu_slab.py \
  > gpurun_out/r3_ck42/tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck42/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck42/tests.txt
for rep in 1 2; do
  for v in e5 e5off; do
    if [ $v = e5 ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    timeout -k 10 300 python bench.py --steps 400 --warmup 40 --legs c2,c2_lap,c2_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck42/$v$rep.json 2>gpurun_out/r3_ck42/$v$rep.err || { tail -20 gpurun_out/r3_ck42/$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck42/$v$rep.json').read().splitlines()[-1])
print('$v rep $rep', ' '.join(f\"{k} {d[k]['it_per_s']} it/s kernel {d[k]['roofline']['kernel_ms']*1e3:.1f} us\" for k in ('c2','c2_lap','c2_cen')))" | tee -a gpurun_out/r3_ck42/ab.txt
  done
done
unset PCS_LIB_PATH
bash tools/r3_ck41.sh
