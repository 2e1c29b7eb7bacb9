"""Per-launch HBM traffic of the fused PDS step from rocprofv3 PMC passes.

Usage: python tools/traffic_from_pmc.py <fetch_csv> <write_csv> <out_json> [kernel_substring]

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads -> doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  The step kernel's global reads are all 16-B-per-lane
group loads in the vectorised layout, its stores 16-B-per-lane group stores.
"""
import csv
import json
import sys


def per_launch(path, counter, kern):
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if r['Counter_Name'] == counter and kern in r['Kernel_Name']]
    if not vals:
        raise SystemExit(f'no {counter} rows for {kern} in {path}')
    # launches that found the loop already stopped move (almost) nothing: average the working ones
    work = [v for v in vals if v >= 0.5 * max(vals)]
    return sum(work) / len(work), len(work)


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    kern = sys.argv[4] if len(sys.argv) > 4 else 'k_pds2d'
    f_kib, nf = per_launch(fetch_csv, 'FETCH_SIZE', kern)
    w_kib, nw = per_launch(write_csv, 'WRITE_SIZE', kern)
    rd = 2.0 * f_kib * 1024
    wr = w_kib * 1024
    res = {'kernel': kern, 'launches': [nf, nw], 'FETCH_SIZE_KiB': f_kib, 'WRITE_SIZE_KiB': w_kib,
           'read_bytes': rd, 'write_bytes': wr, 'traffic_bytes': rd + wr,
           'correction': 'FETCH_SIZE x2 (gfx950, 16-B streaming reads); WRITE_SIZE as reported'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
