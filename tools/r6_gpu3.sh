#!/bin/bash
# Round 6: 3-D parity after the split-half fp64 LDS tiles + the new many-rank slab tests, then the volume legs
set -o pipefail
O=gpurun_out/r6_3; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_pds.py -k "pds3d" \
  tests/test_gpu_slab.py tests/test_gpu_long2.py tests/test_gpu_determinism.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --legs "" --no-cpu-baseline > $O/bench.txt 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r6_3/bench.txt').read().strip().split('\n')[-1])
print('C3', d['value'])
for k in ('volume_c4', 'volume_c5', 'volume_c4_cen', 'volume_c5_cen'):
    v = d.get(k) or {}
    r = v.get('roofline') or {}
    print(k, v.get('it_per_s'), v.get('iteration_frac_of_hbm_peak_per_gpu'), {p: q['kernel_ms'] for p, q in (r.get('parts') or {}).items()})
PY
