#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PCS_ITERS=6
OUT=gpurun_out/abl; mkdir -p $OUT
for m in "$@"; do
  PCS_LIB_PATH=$PWD/scratch/abl/lib$m.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $OUT/m$m -o run --output-format csv -- python3 tools/profile_step.py > $OUT/m$m.log 2>&1 || exit 1
done
echo abl_ok
