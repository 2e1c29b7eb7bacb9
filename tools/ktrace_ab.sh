#!/bin/bash
# Round 5: per-kernel times of a bench run under each env config ($@: "NAME=VAL ..." or "-"); BENCH_ARGS: the
# bench.py arguments; the top kernels of each run's rocprofv3 --stats go to gpurun_out/$OUT/ktrace.txt
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r5_ktrace}
mkdir -p $out
i=0
for cfg in "$@"; do
  i=$((i+1)); envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/t$i -o run --output-format csv -- \
      python3 bench.py $BENCH_ARGS > $out/t$i.log 2>&1 || { echo "FAILED $cfg"; tail -5 $out/t$i.log; exit 1; }
  f=$(find $out/t$i -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$cfg" <<'PY' | tee -a $out/ktrace.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:6]:
    print(sys.argv[2], '%-70s calls=%5s avg_us=%9.2f' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3))
PY
  find $out/t$i -name "*kernel_trace.csv" -delete
done
