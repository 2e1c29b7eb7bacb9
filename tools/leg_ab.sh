#!/bin/bash
# Round 5: 2-D bench legs A/B ($LEGS, default c3_nonsep; $@: "NAME=VAL ..." per run, "-" for the default):
# it/s, iteration fraction and kernel times appended to gpurun_out/$OUT/ab.txt
set -o pipefail
out=gpurun_out/${OUT:-r5_legab}
legs=${LEGS:-c3_nonsep}
mkdir -p $out
for cfg in "$@"; do
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-200} --warmup 20 --legs $legs --volumes "" \
      --no-cpu-baseline > $out/run.json 2> $out/run.err || { echo "FAILED $cfg"; tail -5 $out/run.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/run.json'))
for k in '$legs'.split(','):
    v=d[k]; print('$cfg', k, 'it/s', v.get('it_per_s'), 'ms', v.get('ms_per_iter'), 'frac', v.get('iteration_frac_of_hbm_peak'), v.get('kernels_ms'), v.get('error'))
" | tee -a $out/ab.txt
done
