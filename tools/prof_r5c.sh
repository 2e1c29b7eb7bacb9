#!/bin/bash
# Round-5 PMC / traffic passes after the border-strip split and the GEN race fix (tools/prof_nm.sh per problem)
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c2_lap PCS_ITERS=60 bash tools/prof_nm.sh $1_lap k_pds2d_smarch || exit 1
PCS_PROBLEM=c3_cen bash tools/prof_nm.sh $1_c3cen k_pds2d_nmarch_gen || exit 2
echo prof_r5c_ok
