#!/bin/bash
# PMC passes over tools/ata_probe.py (k_sep2d_nrm, k_sep2d_ata, k_sep2d_march), each its own run
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_nrm
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- python3 tools/ata_probe.py > $OUT/pmc1.log 2>&1 || exit 12
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- python3 tools/ata_probe.py > $OUT/pmc2.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT -d $OUT/pmc3 -o run --output-format csv -- python3 tools/ata_probe.py > $OUT/pmc3.log 2>&1 || echo pmc3_failed
python3 tools/pmc_summary.py "$OUT/pmc*/**/*counter_collection.csv" > $OUT/pmc_summary.txt 2>&1 || true
find $OUT -name "*counter_collection.csv" -delete; find $OUT -name "*agent_info.csv" -delete
cat $OUT/pmc_summary.txt | grep -i -E "nrm|sep2d|kernel|counter" | head -60
