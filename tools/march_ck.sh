# C3 kernel parity (march / nmarch tests) and a bench line
set -o pipefail
mkdir -p gpurun_out/marchck
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_march.py tests/test_gpu_pds.py > gpurun_out/marchck/tests.txt 2>&1 || { tail -30 gpurun_out/marchck/tests.txt; exit 1; }
tail -2 gpurun_out/marchck/tests.txt
timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/marchck/bench.log 2>&1 || { tail -20 gpurun_out/marchck/bench.log; exit 2; }
python3 -c "
import json
d=json.loads(open('gpurun_out/marchck/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])
"
