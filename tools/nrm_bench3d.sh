# C4 / C5 iteration rate with the in-plane normal operator (PCS_3D_ATA=1) against the default
# three-pass gradient, alternating
set -o pipefail
mkdir -p gpurun_out/nrmb
for rep in 1 2; do
  for ata in 0 1; do
    PCS_3D_ATA=$ata timeout -k 10 240 python3 tools/bench3d.py --size 512 --dtype f32 --steps 20 --warmup 4 > gpurun_out/nrmb/c4_${ata}_$rep.json 2>gpurun_out/nrmb/err.txt || { tail -5 gpurun_out/nrmb/err.txt; exit 1; }
    echo "C4 ata=$ata rep $rep: $(cat gpurun_out/nrmb/c4_${ata}_$rep.json)"
  done
done
for ata in 0 1; do
  PCS_3D_ATA=$ata timeout -k 10 300 python3 tools/bench3d.py --size 1024 --dtype f64 --steps 8 --warmup 2 > gpurun_out/nrmb/c5_$ata.json 2>gpurun_out/nrmb/err.txt || { tail -5 gpurun_out/nrmb/err.txt; exit 1; }
  echo "C5 ata=$ata: $(cat gpurun_out/nrmb/c5_$ata.json)"
done
