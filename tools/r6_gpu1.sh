#!/bin/bash
# Round 6, first GPU call: the touched kernels' tests, the C5 centred leg with per-launch rooflines, and what
# processes the bench leaves behind (BENCH r04/r05 procs_at_end: 1).
set -o pipefail
mkdir -p gpurun_out/r6_1
O=gpurun_out/r6_1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_nm64.py \
  > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs conv63 --no-cpu-baseline \
  --volumes c5_cen:1024:f64:20:centered,c4:512:f32:20 > $O/bench.txt 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
sleep 2
ps -u "$(id -u)" -o pid,ppid,etime,stat,cmd > $O/ps_after.txt
cat $O/ps_after.txt
python - <<'EOF'
import json
d = json.loads(open('gpurun_out/r6_1/bench.txt').read().strip().split('\n')[-1])
for k in ('volume_c5_cen', 'volume_c4'):
    print(k, json.dumps(d.get(k))[:1500])
EOF
