#!/bin/bash
# Profile the fused step on the GPU box: kernel-trace stats + separate PMC passes.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r1}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/profile_step.py > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- python3 tools/profile_step.py > $OUT/pmc1.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- python3 tools/profile_step.py > $OUT/pmc2.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 tools/profile_step.py > $OUT/pmc3.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o run --output-format csv -- python3 tools/profile_step.py > $OUT/pmc4.log 2>&1 || exit 15
echo prof_ok
