#!/bin/bash
# Round 5: C3 centred determinism after the LDS-DMA wait fix (tools/det_probe.py) + the nmarch tests + bench legs
set -o pipefail
out=gpurun_out/${OUT:-r5_det2}
mkdir -p $out
PROBS=c3_cen timeout -k 10 400 python tools/det_probe.py > $out/det.txt 2>&1 || exit 1
grep iters $out/det.txt
