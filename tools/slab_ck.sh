# multi-slab parity tests + a short bench line (N=1)
set -o pipefail
mkdir -p gpurun_out/slabck
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_slab.py > gpurun_out/slabck/tests.txt 2>&1 || { tail -30 gpurun_out/slabck/tests.txt; exit 1; }
tail -2 gpurun_out/slabck/tests.txt
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/slabck/bench.log 2>&1 || { tail -20 gpurun_out/slabck/bench.log; exit 2; }
python3 -c "
import json
d=json.loads(open('gpurun_out/slabck/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['volume_c4'], d['volume_c5'])
"
