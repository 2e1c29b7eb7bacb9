#!/bin/bash
# round-2: the 2-D legs of bench.py alone (no headline cpu baseline, no volumes) + kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-legs}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --volumes "" ${LEGS_ARGS} > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
python3 - <<PY
import csv,glob
f=glob.glob('$O/prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'pcs' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,1),'us')
PY
find $O/prof -name '*kernel_trace.csv' -delete
