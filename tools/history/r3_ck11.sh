#!/bin/bash
# round 3 checkpoint 11: PMC traffic + SQ counters of k_pds3d_gen (C4 centred), k_corr2d,
# k_pds2d_gen (lap / cen, PCS_STENCIL_MARCH=0) and the c3_cen pair
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof3d.sh r3_cen 512 f32 centered || exit $?
cat gpurun_out/prof3d_r3_cen/pmc_summary.txt | head -60
PCS_PROBLEM=c3_nonsep bash tools/prof_nm.sh r3_prof_corr k_corr2d || exit $?
PCS_STENCIL_MARCH=0 PCS_PROBLEM=c2_lap bash tools/prof_nm.sh r3_prof_gen_lap k_pds2d_gen || exit $?
PCS_STENCIL_MARCH=0 PCS_PROBLEM=c2_cen bash tools/prof_nm.sh r3_prof_gen_cen k_pds2d_gen || exit $?
PCS_PROBLEM=c3_cen bash tools/prof_nm.sh r3_prof_c3cen k_pds2d_smarch || exit $?
for d in r3_prof_corr r3_prof_gen_lap r3_prof_gen_cen r3_prof_c3cen; do echo "== $d"; cat gpurun_out/$d/traffic.json | tr -d '\n'; echo; done
