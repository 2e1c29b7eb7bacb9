# general-stencil step: parity tests, then the bench's c2_lap / c2_cen legs (default build and the
# given variants: tools/build_var.sh NAME ...)
set -o pipefail
mkdir -p gpurun_out/gen
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stencil.py tests/test_gpu_pds.py > gpurun_out/gen/tests.txt 2>&1 || { tail -30 gpurun_out/gen/tests.txt; exit 1; }
tail -2 gpurun_out/gen/tests.txt
for v in default "$@"; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/gen/bench_$v.log 2>&1 || { tail -20 gpurun_out/gen/bench_$v.log; exit 2; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/gen/bench_$v.log').read().strip().splitlines()[-1])
print('$v', 'C3', d['value'], 'lap', d['c2_lap']['roofline']['kernel_ms'], d['c2_lap']['it_per_s'], 'cen', d['c2_cen']['roofline']['kernel_ms'], d['c2_cen']['it_per_s'])
"
done
