#!/bin/bash
# Round 6: 3-D slabs after the z-halo trim (bitwise), C5/8 rank share + link-rate model (forward, centred),
# LDS bank conflicts of the C5 update kernels after the split-half fp64 tiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_6; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_slab.py -k "3d or pds3d or vol" \
  > $O/slab3d.txt 2>&1 || { echo "slab3d tests failed"; grep -E "^E |FAILED" $O/slab3d.txt | head; exit 1; }
tail -2 $O/slab3d.txt
timeout -k 10 300 python -u tools/bench3d.py --size 1024 --dtype f64 --rank-of 8 --steps 16 --one-gpu-ms 24.3 > $O/share_c5.txt 2>&1 || { echo "share c5 failed"; tail $O/share_c5.txt; exit 1; }
tail -1 $O/share_c5.txt
timeout -k 10 300 python -u tools/bench3d.py --size 1024 --dtype f64 --rank-of 8 --steps 16 --kind centered --one-gpu-ms 28.5 > $O/share_c5cen.txt 2>&1 || { echo "share c5cen failed"; tail $O/share_c5cen.txt; exit 1; }
tail -1 $O/share_c5cen.txt
cd /tmp
for k in c4 c4_cen; do
  PCS_PROBLEM=$k PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=3 timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/$O/pmc_$k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/profile_step.py > $GRAFT_REPO_ROOT/$O/pmc_$k.log 2>&1 || { echo "pmc $k failed"; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py "$O/pmc_*/**/*counter_collection.csv" > $O/pmc_summary.txt 2>&1 || true
grep -A6 "k_pds3d" $O/pmc_summary.txt | head -30
find $O -name "*counter_collection.csv" -delete
echo ok
