#!/bin/bash
# Round-4 PMC passes on the final kernels: fp64 C3 (grad F formed in the N x pass: k_sep2d_nrm<double, true>
# + the GRADBUF march step), the 2048^2 Laplacian march
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c3 PCS_DTYPE=f64 bash tools/prof_nm.sh $1_c3f64 k_pds2d_smarch || exit 1
PCS_PROBLEM=c2_lap bash tools/prof_nm.sh $1_lap k_pds2d_smarch || exit 2
echo prof_r4b_ok
