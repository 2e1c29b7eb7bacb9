#!/bin/bash
# Round-4 PMC / traffic passes (tools/prof_nm.sh per problem): the shipped C3 kernel (the bench line's
# roofline.traffic), the fp64 C3 march step + N x pass, the fused CPS inpainting step
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c3 bash tools/prof_nm.sh $1_c3 k_pds2d_nmarch || exit 1
PCS_PROBLEM=c3 PCS_DTYPE=f64 bash tools/prof_nm.sh $1_c3f64 k_pds2d_smarch || exit 2
PCS_PROBLEM=cps bash tools/prof_nm.sh $1_cps k_pds2d_smarch || exit 3
PCS_PROBLEM=c4_cen PCS_ITERS=8 bash tools/prof_nm.sh $1_c4cen k_pds3d_gen || exit 4
echo prof_r4_ok
