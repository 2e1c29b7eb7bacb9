#!/bin/bash
# Round-5 PMC / traffic passes (tools/prof_nm.sh per problem): the fused fp64 C3 march (forward and the
# default centred K) and the C5 fp64 3-D iteration (its in-plane normal operator k_sep2d_nrmm)
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c3 PCS_DTYPE=f64 bash tools/prof_nm.sh $1_c3f64 k_pds2d_nmarch64 || exit 1
PCS_PROBLEM=c3_cen PCS_DTYPE=f64 bash tools/prof_nm.sh $1_c3cenf64 k_pds2d_nmarch64 || exit 2
PCS_PROBLEM=c4 PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=6 bash tools/prof_nm.sh $1_c5 k_sep2d_nrmm || exit 3
echo prof_r5_ok
