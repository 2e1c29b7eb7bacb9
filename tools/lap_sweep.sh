#!/bin/bash
# Round 5: the stencil march's fixed cost -- tools/sm_probe.py (Laplacian / centred K denoising) over image
# sizes and PCS_SM_SLOTS grids; JSON lines appended to gpurun_out/$OUT/sweep.txt
set -o pipefail
out=gpurun_out/${OUT:-r5_lap}
mkdir -p $out
for n in 1024 2048 3072 4096; do
  PCS_N=$n timeout -k 10 120 python -u tools/sm_probe.py 2>>$out/err.txt | sed "s/^/n=$n slots=default /" | tee -a $out/sweep.txt
done
for s in 256 512 1024 1536 2048; do
  PCS_N=2048 PCS_SM_SLOTS=$s timeout -k 10 120 python -u tools/sm_probe.py 2>>$out/err.txt | sed "s/^/n=2048 slots=$s /" | tee -a $out/sweep.txt
done
