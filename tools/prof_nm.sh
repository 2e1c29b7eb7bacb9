#!/bin/bash
# Profile the C3 fused step (tools/profile_step.py): kernel trace + PMC passes (each its own run)
# + per-launch HBM traffic of the step kernel.  $1: output dir under gpurun_out/, $2: kernel name substring.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof_nm}; K=${2:-k_pds2d_nmarch}; PY=${PCS_PROF_PY:-tools/profile_step.py}  # PCS_PROF_PY: another driver script
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $PY > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- python3 $PY > $OUT/pmc1.log 2>&1 || exit 12
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- python3 $PY > $OUT/pmc2.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 $PY > $OUT/pmc3.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o run --output-format csv -- python3 $PY > $OUT/pmc4.log 2>&1 || exit 15
f3=$(find $OUT/pmc3 -name '*counter_collection.csv' | head -1); f4=$(find $OUT/pmc4 -name '*counter_collection.csv' | head -1)
python3 tools/traffic_from_pmc.py $f3 $f4 $OUT/traffic.json $K > /dev/null || exit 16
python3 tools/pmc_summary.py "$OUT/pmc*/**/*counter_collection.csv" > $OUT/pmc_summary.txt 2>&1 || true
find $OUT -name "*kernel_trace.csv" -delete; find $OUT -name "*counter_collection.csv" -delete; find $OUT -name "*agent_info.csv" -delete
echo prof_ok
