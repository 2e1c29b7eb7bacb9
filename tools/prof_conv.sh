#!/bin/bash
# PMC passes over the standalone Convolve2D kernel (tools/conv2d_bench.py, 4096^2, k=15 fp32).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_conv_${1:-r2}
mkdir -p $OUT
CMD="python3 tools/conv2d_bench.py --ks ${2:-15} --dtypes ${3:-f32} --iters 20"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || exit 11
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- $CMD > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- $CMD > $OUT/pmc2.log 2>&1 || exit 13
python3 tools/pmc_summary.py "$OUT/pmc*/*/*counter_collection.csv" "$OUT/pmc*/*counter_collection.csv" > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
grep -h corr2d $OUT/trace/*kernel_stats.csv $OUT/trace/*/*kernel_stats.csv 2>/dev/null | head -5
echo prof_ok
