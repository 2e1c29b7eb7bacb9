#!/bin/bash
# round 3 checkpoint 6: slab engine generality (in-process + two-process gloo), FFT + smarch parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_smarch.py tests/test_gpu_fftconv.py tests/test_gpu_stencil.py > gpurun_out/r3_ck6_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r3_ck6_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for bl in 2048 1024 0; do
  PCS_FFT_BLOCK=$bl timeout -k 10 200 python bench.py --steps 50 --warmup 5 --legs conv63 --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck6_fft_b$bl.json 2>/dev/null || exit $?
done
# A/B: plain vs sc1 (write-through) x' / z' stores in the pt (C2) and nmarch (C3) kernels, alternating
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 500 --warmup 50 --legs c2 --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck6_ab_plain_$i.json 2>/dev/null || exit $?
  PCS_LIB_PATH=pycsou_amd/lib/var/sc1all/libpycsou_hip.so timeout -k 10 300 python bench.py --steps 500 --warmup 50 --legs c2 --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck6_ab_sc1_$i.json 2>/dev/null || exit $?
done
