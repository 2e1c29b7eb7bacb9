"""Average PMC counters per kernel (name substring filter) from rocprofv3 counter CSVs.
Usage: python tools/pmc_kernels.py SUBSTR 'gpurun_out/x/pmc*/*counter_collection.csv' ..."""
import collections
import csv
import glob
import sys

sub = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for pat in sys.argv[2:]:
    for f in glob.glob(pat):
        for r in csv.DictReader(open(f)):
            if sub in r['Kernel_Name']:
                vals[r['Kernel_Name'][:70]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})')
