#!/bin/bash
# round 3 checkpoint 18: PMC of the C4 loop with the default centred K (16-row k_pds3d_gen) and forward K
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof3d.sh r3_cen16 512 f32 centered || exit $?
bash tools/prof3d.sh r3_fwd 512 f32 forward || exit $?
for d in r3_cen16 r3_fwd; do echo "== $d"; grep -A17 "k_pds3d" gpurun_out/prof3d_$d/pmc_summary.txt | head -40; done
