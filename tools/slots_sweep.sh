#!/bin/bash
# Round 5: grid-size (slots) re-sweep after deferred finalization -- $@: "VAR=v1,v2,...:legs" specs; every
# value runs bench.py (C3 headline + the given legs) in its own process (the knobs are read once)
set -o pipefail
out=gpurun_out/${OUT:-r5_slots}
mkdir -p $out
for spec in "$@"; do
  var=${spec%%=*}; rest=${spec#*=}; vals=${rest%%:*}; legs=${rest#*:}
  for v in ${vals//,/ }; do
    if [ "$v" = def ]; then E=PCS_X=0; else E=$var=$v; fi
    env $E timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --legs $legs --volumes "" --no-cpu-baseline \
        > $out/run.json 2>> $out/err.txt || exit 2
    python -c "
import json; d=json.load(open('$out/run.json'))
print('$var=$v', 'C3', d['value'], {k: v.get('it_per_s') for k, v in d.items() if isinstance(v, dict) and 'it_per_s' in v})" | tee -a $out/sweep.txt
  done
done
