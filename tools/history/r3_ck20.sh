#!/bin/bash
# round 3 checkpoint 20: k_pds3d_gen fp32 tile rows 16 (default) vs 8 (tools/build_var.sh g3r8 -DPCS_3DG_ROWS32=8)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default g3r8 default g3r8; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  echo -n "$v "; timeout -k 10 200 python tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4 --kind centered 2>/dev/null | tail -1 || exit $?
done
