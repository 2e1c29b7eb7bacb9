#!/bin/bash
# Round-5 PMC / traffic passes after the deferred finalization (tools/prof_nm.sh per problem): C3 (k_pds2d_nmarch),
# the 2048^2 Laplacian and centred stencil marches, C2 (k_pds2d_pt) and the CPS masked march
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c3 bash tools/prof_nm.sh $1_c3 k_pds2d_nmarch || exit 1
PCS_PROBLEM=c2_lap PCS_ITERS=60 bash tools/prof_nm.sh $1_lap k_pds2d_smarch || exit 2
PCS_PROBLEM=c2 PCS_ITERS=60 bash tools/prof_nm.sh $1_c2 k_pds2d_pt || exit 3
PCS_PROBLEM=cps PCS_ITERS=60 bash tools/prof_nm.sh $1_cps k_pds2d_smarch || exit 4
echo prof_r5b_ok
