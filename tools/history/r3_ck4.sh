#!/bin/bash
# round 3 checkpoint 4: smarch two-set prefetch (parity + legs), FFT grid probe with kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_smarch.py tests/test_gpu_stencil.py > gpurun_out/r3_ck4_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r3_ck4_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --legs c2_lap,c2_cen,c3_cen --volumes "" --no-cpu-baseline > gpurun_out/r3_ck4_bench.json 2> gpurun_out/r3_ck4_bench.err || exit $?
for g in 4200 4160 4320 4374 4608 5120; do
  PCS_FFT_GRID=$g timeout -k 10 200 python bench.py --steps 50 --warmup 5 --legs conv63 --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck4_fft_$g.json 2>/dev/null || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_ck4_fft_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --legs conv63 --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck4_fft_trace.log 2>&1 || exit $?
find gpurun_out/r3_ck4_fft_trace -name "*kernel_trace.csv" -delete
