# C4 A/B: tools/bench3d.py with the default build and a variant (tools/build_var.sh NAME), alternating
set -o pipefail
mkdir -p gpurun_out/c4ab
for rep in 1 2; do
  for v in default "$1"; do
    if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
    timeout -k 10 200 python3 tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4 > gpurun_out/c4ab/${v}_$rep.txt 2>&1 || { tail -5 gpurun_out/c4ab/${v}_$rep.txt; exit 1; }
    echo "$v rep $rep: $(grep -o '"it_per_s": [0-9.]*, "ms_per_iter": [0-9.]*, "update_kernel_ms": [0-9.]*' gpurun_out/c4ab/${v}_$rep.txt)"
  done
done
