#!/bin/bash
# round 6: fp64 march border strips on a row-interior form (in-tree) vs the all-axes edge form (var nm64rf0).
# fp64 march tests, then the c3_f64 / c3_cen_f64 legs, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_nm64rf; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_nm64.py tests/test_gpu_determinism.py \
  tests/test_gpu_fullsize.py -k "nm64 or f64 or float64 or determin" > $O/tests.txt 2>&1 || { grep -E "^E |FAILED" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in default nm64rf0; do
    if [ $v = default ]; then L=""; else L=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    PCS_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --legs c3_f64,c3_cen_f64 --volumes "" --no-cpu-baseline > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/run.json'))
for k in ('c3_f64','c3_cen_f64'):
    v=d[k]; print('$v rep$r', k, 'it/s', v.get('it_per_s'), 'frac', v.get('iteration_frac_of_hbm_peak'), v.get('kernels_ms'))
" | tee -a $O/ab.txt
  done
done
