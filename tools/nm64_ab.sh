#!/bin/bash
# Round 5: fused fp64 march A/B -- bench legs c3_f64 / c3_cen_f64 under env settings ($@: "NAME=VAL ..." per
# run, "-" for the default), results in gpurun_out/$OUT/ab.txt
set -o pipefail
out=gpurun_out/${OUT:-r5_nm64ab}
mkdir -p $out
for cfg in "$@"; do
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --legs c3_f64,c3_cen_f64 --volumes "" \
      --no-cpu-baseline > $out/run.json 2> $out/run.err || { echo "FAILED $cfg"; tail -5 $out/run.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/run.json'))
for k in ('c3_f64','c3_cen_f64'):
    v=d[k]; print('$cfg', k, 'it/s', v['it_per_s'], 'ms', v['ms_per_iter'], 'frac', v['iteration_frac_of_hbm_peak'], v.get('kernels_ms'))
" | tee -a $out/ab.txt
done
