#!/bin/bash
# Round 5: k_pds3d_gen edge-path A/B on the C4 centred problem (tools/bench3d.py, 512^3 fp32) -- kernel trace
# per library; $@: "default" or variant names under pycsou_amd/lib/var/
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r5_g3d}
mkdir -p $out
for v in "$@"; do
  if [ "$v" = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$v -o run --output-format csv -- python3 tools/bench3d.py --kind ${KIND:-centered} --size ${SIZE:-512} --steps 20 > $out/$v.log 2>&1 || exit 1
  python3 - $out/$v $v <<'PY' | tee -a $out/ab.txt
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'pcs::' in r['Name']]
print(sys.argv[2], {r['Name'].split('(')[0].replace('void pcs::', '')[:40]: round(float(r['AverageNs']) / 1e3, 1) for r in rows
                    if float(r['TotalDurationNs']) > 1e6})
PY
  tail -1 $out/$v.log | tee -a $out/ab.txt
  find $out/$v -name '*kernel_trace.csv' -delete
done
