#!/bin/bash
# Round 5: k_corr2d_mf ablation timings (tools/conv2d_bench.py 4096^2 k = 15 fp32) for the default library, the
# VALU kernel and the variant builds pycsou_amd/lib/var/$v (tools/build_var.sh), -> gpurun_out/$OUT/abl.txt
set -o pipefail
out=gpurun_out/${OUT:-r5_mfabl}
mkdir -p $out
run() { echo -n "$1 " | tee -a $out/abl.txt; shift; env "$@" timeout -k 10 120 python3 tools/conv2d_bench.py --ks 15 --dtypes f32 --iters 50 2>>$out/err.txt | tee -a $out/abl.txt || exit 1; }
run default PCS_X=0
run valu PCS_CORR_MFMA=0
for v in "$@"; do run $v PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; done
