#!/bin/bash
# round 3 checkpoint 39: folded C4 kernel with 2-voxel ring items on waves 6-15 (PCS_3D_RV=2) and the ring
# prologue's loads 4 planes ahead (PCS_3D_RPD=4): 3-D fold / slab parity, then C4 A/B against the
# previous form (RV=3, RPD=1) and RV=2 alone, alternating
set -o pipefail
mkdir -p gpurun_out/r3_ck39
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pds.py tests/test_gpu_slab.py -k "3d or folded" \
  > gpurun_out/r3_ck39/tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck39/tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck39/tests.txt
for rep in 1 2; do
  for v in new old3d rv2pd1; do
    if [ $v = new ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck39/$v$rep.json 2>gpurun_out/r3_ck39/$v$rep.err || { tail -20 gpurun_out/r3_ck39/$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck39/$v$rep.json').read().splitlines()[-1]); c=d['volume_c4']
print('$v rep $rep', c['it_per_s'], c['ms_per_iter'])" | tee -a gpurun_out/r3_ck39/ab.txt
  done
done
