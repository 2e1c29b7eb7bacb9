#!/bin/bash
# PMC passes over the 3-D C4 loop (tools/bench3d.py): HBM traffic + SQ counters per kernel.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out/prof3d_${1:-r1}
SZ=${2:-512}
DT=${3:-f32}
mkdir -p $OUT
cd /tmp || exit 1
KIND=${4:-forward}
P="python3 $R/tools/bench3d.py --size $SZ --dtype $DT --steps 6 --warmup 2 --kind $KIND"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $P > $OUT/pmc1.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc2 -o run --output-format csv -- $P > $OUT/pmc2.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/pmc3 -o run --output-format csv -- $P > $OUT/pmc3.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc4 -o run --output-format csv -- $P > $OUT/pmc4.log 2>&1 || exit 15
python3 $R/tools/pmc_summary.py "$OUT/pmc*/**/*counter_collection.csv" > $OUT/pmc_summary.txt 2>&1 || true
find $OUT -name "*counter_collection.csv" -delete; find $OUT -name "*agent_info.csv" -delete
echo prof3d_ok
