#!/bin/bash
# round 3 checkpoint 27: axis-0 pass folded into the 3-D update (PCS_F_CONV0): tests, then C4 with / without
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pds.py -k "pds3d" \
  > gpurun_out/r3_ck27_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck27_tests.txt; exit 1; }
tail -2 gpurun_out/r3_ck27_tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_slab.py -k "3d" \
  > gpurun_out/r3_ck27_slab_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck27_slab_tests.txt; exit 1; }
tail -2 gpurun_out/r3_ck27_slab_tests.txt
for f in 1 0 1 0; do
  PCS_3D_FOLD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck27_fold$f.json 2>gpurun_out/r3_ck27_fold$f.err || { tail -20 gpurun_out/r3_ck27_fold$f.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck27_fold$f.json').read().splitlines()[-1]); c=d['volume_c4']
print('fold $f', c['it_per_s'], c['ms_per_iter'])"
done
