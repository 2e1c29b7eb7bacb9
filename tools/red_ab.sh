#!/bin/bash
# Round 5: in-kernel reduction A/B -- the stencil march (tools/sm_probe.py, 2048^2 Laplacian / centred) and the
# C3 / C2 bench legs under each library ($@: "default" or a variant name under pycsou_amd/lib/var/)
set -o pipefail
out=gpurun_out/${OUT:-r5_redab}
mkdir -p $out
for v in "$@"; do
  if [ "$v" = default ]; then E=PCS_X=0; else E=PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  env $E PCS_N=2048 timeout -k 10 120 python3 tools/sm_probe.py 2>>$out/err.txt | sed "s|^|$v |" | tee -a $out/ab.txt || exit 1
  env $E timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --legs c2,cps_inpaint --volumes "" --no-cpu-baseline \
      > $out/run.json 2>> $out/err.txt || exit 2
  python -c "
import json; d=json.load(open('$out/run.json'))
print('$v', 'C3', d['value'], 'c2', d['c2']['it_per_s'], 'cps', d['cps_inpaint']['it_per_s'])" | tee -a $out/ab.txt
done
