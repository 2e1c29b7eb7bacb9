#!/bin/bash
# Round 6: PMC of the C5 (1024^3 fp64) update kernels -- the default centred K (k_pds3d_gen<double>) and
# the forward K (k_pds3d<double>) for comparison
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c4_cen PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 bash tools/prof_nm.sh r6_c5cen k_pds3d_gen || exit 1
PCS_PROBLEM=c4 PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 bash tools/prof_nm.sh r6_c5fwd k_pds3d || exit 2
echo r6_prof_c5_ok
