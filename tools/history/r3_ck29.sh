#!/bin/bash
# round 3 checkpoint 29: folded axis-0 pass, rings on the U-item waves; C4 timing A/B with diagnostic
# variants (tools: pycsou_amd/lib/var/fdN = -DPCS_3D_FOLD_DIAG=N: 1 no shifts, 2 no sums, 4 no prologue)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pds.py -k "folded" \
  > gpurun_out/r3_ck29_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck29_tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck29_tests.txt
for v in fold0 fold1 fd1 fd2 fd4 fd3 fold1 fold0; do
  unset PCS_LIB_PATH; export PCS_3D_FOLD=1
  case $v in fold0) export PCS_3D_FOLD=0;; fold1) ;; *) export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so;; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck29_$v.json 2>gpurun_out/r3_ck29_$v.err || { tail -20 gpurun_out/r3_ck29_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck29_$v.json').read().splitlines()[-1]); c=d['volume_c4']
print('$v', c['it_per_s'], c['ms_per_iter'])"
done
unset PCS_LIB_PATH; export PCS_3D_FOLD=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_ck29_prof -o run -- python3 bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck29_prof.log 2>&1 || { tail -20 gpurun_out/r3_ck29_prof.log; exit 1; }
f=$(find gpurun_out/r3_ck29_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3_ck29_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r3_ck29_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
PY
