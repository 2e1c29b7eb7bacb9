set -o pipefail
bash tools/r2_stencil.sh st2 && LEGS_ARGS="--legs c2,c2_lap,c2_cen --lipschitz analytic" bash tools/r2_legs.sh legs2
