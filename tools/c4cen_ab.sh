#!/bin/bash
# Round 5: C4 volume legs A/B ($@: "NAME=VAL ..." per run, "-" for the default): volume_c4 and volume_c4_cen
# it/s and kernel times, results appended to gpurun_out/$OUT/ab.txt
set -o pipefail
out=gpurun_out/${OUT:-r5_c4ab}
mkdir -p $out
for cfg in "$@"; do
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs "" \
      --volumes ${VOLS:-c4:512:f32:20,c4_cen:512:f32:20:centered} --no-cpu-baseline > $out/run.json 2> $out/run.err \
      || { echo "FAILED $cfg"; tail -5 $out/run.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/run.json'))
for k, v in d.items():
    if k.startswith('volume_') and isinstance(v, dict):
        print('$cfg', k, {q: v.get(q) for q in ('it_per_s', 'ms_per_iter', 'iteration_frac_of_hbm_peak_per_gpu', 'axis0_folded', 'error')})
" | tee -a $out/ab.txt
done
