#!/bin/bash
# kernel-trace stats of the eager C3 engine (tools/profile_step.py)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ktrace_${1:-x}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/profile_step.py > $OUT/log.txt 2>&1 || exit 11
python3 -c "
import csv,glob
f=glob.glob('$OUT/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1),'us')
"
