#!/bin/bash
# round-2: k_sep2d_ata parity + 3-D engine tests + volume bench legs + kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-ata}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "ata or conv0 or sep_planes" -x -q --timeout 120 --timeout-method thread > $O/t_ops.txt 2>&1 || { echo OPS_FAILED; tail -40 $O/t_ops.txt; exit 1; }
tail -2 $O/t_ops.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pds.py tests/test_gpu_slab.py -k "3d or 3D or volume or slab3d" -x -q --timeout 120 --timeout-method thread > $O/t_3d.txt 2>&1 || { echo T3D_FAILED; tail -40 $O/t_3d.txt; exit 2; }
tail -2 $O/t_3d.txt
timeout -k 10 300 python3 tools/bench3d.py --size 512 --dtype f32 > $O/bench3d_c4.log 2>&1 || { echo B3D_FAILED; tail -30 $O/bench3d_c4.log; exit 3; }
tail -2 $O/bench3d_c4.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench3d.py --size 1024 --dtype f64 --steps 10 > $O/bench3d_c5.log 2>&1 || { echo B3D5_FAILED; tail -30 $O/bench3d_c5.log; exit 4; }
tail -2 $O/bench3d_c5.log
python3 - <<PY
import csv,glob
f=glob.glob('$O/prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'pcs' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,1),'us')
PY
