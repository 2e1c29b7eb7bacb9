#!/bin/bash
# round 3 checkpoint 9: generic-path bench leg; PMC traffic of k_corr2d, k_pds2d_gen (lap / cen),
# and the c3_cen pair (k_pds2d_smarch NB + k_sep2d_nrm)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --legs cps_inpaint --volumes "" --no-cpu-baseline --lipschitz analytic > gpurun_out/r3_ck9_cps.json 2> gpurun_out/r3_ck9_cps.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r3_ck9_cps.json').read().splitlines()[-1]); print(d['cps_inpaint'])"
PCS_PROBLEM=c3_nonsep bash tools/prof_nm.sh r3_prof_corr k_corr2d || exit $?
PCS_STENCIL_MARCH=0 PCS_PROBLEM=c2_lap bash tools/prof_nm.sh r3_prof_gen_lap k_pds2d_gen || exit $?
PCS_STENCIL_MARCH=0 PCS_PROBLEM=c2_cen bash tools/prof_nm.sh r3_prof_gen_cen k_pds2d_gen || exit $?
PCS_PROBLEM=c3_cen bash tools/prof_nm.sh r3_prof_c3cen k_pds2d_smarch || exit $?
for d in r3_prof_corr r3_prof_gen_lap r3_prof_gen_cen r3_prof_c3cen; do echo "== $d"; cat gpurun_out/$d/traffic.json | tr -d '\n'; echo; done
