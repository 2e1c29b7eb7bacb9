# k_sep2d_nrm ablation builds (tools/build_var.sh NAME -DPCS_NRM_ABL=bits) timed by ata_probe.py
set -o pipefail
mkdir -p gpurun_out/nrmabl
for v in default "$@"; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  echo "== $v" >> gpurun_out/nrmabl/out.txt
  timeout -k 10 120 python3 tools/ata_probe.py >> gpurun_out/nrmabl/out.txt 2>&1 || { echo FAIL $v; tail -5 gpurun_out/nrmabl/out.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/nrmabl/out.txt
