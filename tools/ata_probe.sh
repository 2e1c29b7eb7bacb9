set -o pipefail
mkdir -p gpurun_out/ataprobe
for v in default rb4 hreg rb4h; do
  if [ $v = default ]; then unset PCS_LIB_PATH; else export PCS_LIB_PATH=$PWD/pycsou_amd/lib/var/$v/libpycsou_hip.so; fi
  timeout -k 10 120 python3 tools/ata_probe.py >> gpurun_out/ataprobe/out.txt 2>&1 || { echo FAIL $v; tail -5 gpurun_out/ataprobe/out.txt; exit 1; }
done
cat gpurun_out/ataprobe/out.txt
