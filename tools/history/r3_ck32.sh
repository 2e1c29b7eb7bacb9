#!/bin/bash
# round 3 checkpoint 31: folded axis-0 pass on dedicated ring waves, ring loop unrolled by 15; C4 A/B + kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pds.py -k "folded" \
  > gpurun_out/r3_ck32_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck32_tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck32_tests.txt
PCS_3D_FOLD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_slab.py -k "3d" \
  > gpurun_out/r3_ck32_slab_tests.txt 2>&1 || { tail -30 gpurun_out/r3_ck32_slab_tests.txt; exit 1; }
tail -1 gpurun_out/r3_ck32_slab_tests.txt
for v in 0 1 0 1; do
  PCS_3D_FOLD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck32_fold$v.json 2>gpurun_out/r3_ck32_fold$v.err || { tail -20 gpurun_out/r3_ck32_fold$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck32_fold$v.json').read().splitlines()[-1]); c=d['volume_c4']
print('fold $v', c['it_per_s'], c['ms_per_iter'])"
done
PCS_3D_FOLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_ck32_prof -o run -- python3 bench.py --steps 20 --warmup 5 --legs "" --volumes c4:512:f32:20 --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck32_prof.log 2>&1 || { tail -20 gpurun_out/r3_ck32_prof.log; exit 1; }
f=$(find gpurun_out/r3_ck32_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3_ck32_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r3_ck32_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:4]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
PY
