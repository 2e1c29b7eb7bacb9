#!/bin/bash
# round 6: PMC traffic of the 3-D general-K updates after the tile changes (C4 centred fp32 12 x 256, C5 centred
# fp64 12 x 128) and of the fp64 forward update (12 rows)
set -o pipefail
export TMPDIR=/tmp
PCS_PROBLEM=c4_cen PCS_DTYPE=f32 PCS_N=512 PCS_ITERS=6 bash tools/prof_nm.sh r6_tiles_c4cen k_pds3d_gen || exit 1
PCS_PROBLEM=c4_cen PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 bash tools/prof_nm.sh r6_tiles_c5cen k_pds3d_gen || exit 2
PCS_PROBLEM=c4 PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 bash tools/prof_nm.sh r6_tiles_c5fwd k_pds3d || exit 3
echo tiles_prof_ok
