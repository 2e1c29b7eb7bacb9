#!/bin/bash
# Round 5: deferred finalization A/B (PCS_DEFER_FIN=1, the default, against 0: the in-launch reduction) --
# the stencil march probe (tools/sm_probe.py) and the 2-D bench legs; $@: the settings to run, in order
set -o pipefail
out=gpurun_out/${OUT:-r5_defer}
mkdir -p $out
for v in "$@"; do
  PCS_DEFER_FIN=$v PCS_N=2048 timeout -k 10 120 python3 tools/sm_probe.py 2>>$out/err.txt | sed "s|^|defer=$v |" | tee -a $out/ab.txt || exit 1
  PCS_DEFER_FIN=$v timeout -k 10 400 python -u bench.py --steps 300 --warmup 30 --legs ${LEGS:-c2,c2_lap,cps_inpaint,c3_cen,c3_f64} \
      --volumes "" --no-cpu-baseline > $out/run_$v.json 2>> $out/err.txt || exit 2
  python -c "
import json; d=json.load(open('$out/run_$v.json'))
print('defer=$v', 'C3', d['value'], {k: v.get('it_per_s') for k, v in d.items() if isinstance(v, dict) and 'it_per_s' in v})" | tee -a $out/ab.txt
done
