#!/bin/bash
# Round 5: PMC passes over the 4096^2 fp32 k = 15 Convolve2D (tools/conv2d_bench.py): MFMA pipe busy, wave
# waits, LDS -- the matrix-core correlation k_corr2d_mf (env: PCS_CORR_MF_SLOTS etc. pass through)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5_prof_mf}
mkdir -p $OUT
CMD="python3 tools/conv2d_bench.py --ks 15 --dtypes f32 --iters 20"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || exit 11
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- $CMD > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- $CMD > $OUT/pmc2.log 2>&1 || exit 13
python3 tools/pmc_summary.py "$OUT/pmc*/*/*counter_collection.csv" "$OUT/pmc*/*counter_collection.csv" > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -delete
echo prof_ok
