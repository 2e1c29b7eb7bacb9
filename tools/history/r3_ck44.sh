#!/bin/bash
# round 3 checkpoint 44: stencil march lands step 0's z rows with the prologue's (PCS_SM_ZEARLY=1):
# smarch / slab / pds parity, then the 2-D stencil legs A/B against landing them at step 0's top
set -o pipefail
mkdir -p gpurun_out/r3_ck44
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_smarch.py tests/test_gpu_slab.py tests/test_gpu_pds.py \
  > gpurun_out/r3_ck44/tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck44/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck44/tests.txt
for rep in 1 2; do
  for v in ze ze0; do
    if [ $v = ze ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    timeout -k 10 300 python bench.py --steps 400 --warmup 40 --legs c2_lap,c2_cen --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck44/$v$rep.json 2>gpurun_out/r3_ck44/$v$rep.err || { tail -20 gpurun_out/r3_ck44/$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck44/$v$rep.json').read().splitlines()[-1])
print('$v rep $rep', ' '.join(f\"{k} {d[k]['it_per_s']} it/s kernel {d[k]['roofline']['kernel_ms']*1e3:.1f} us\" for k in ('c2_lap','c2_cen')))" | tee -a gpurun_out/r3_ck44/ab.txt
  done
done
