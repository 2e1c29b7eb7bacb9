"""Average PMC counters per kernel from rocprofv3 counter_collection CSVs."""
import csv, sys, collections, glob
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for f in glob.glob(path, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'][:60]
            vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in vals.items():
    if not any(t in k for t in ('k_pds', 'reduce', 'conv', 'grad', 'corr', 'sep2d')):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})')
