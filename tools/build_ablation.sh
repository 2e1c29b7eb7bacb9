#!/bin/bash
# Build diagnostic variants of the engine with phases of the fused kernel disabled.
cd "$(dirname "$0")/.." || exit 1
mkdir -p scratch/abl
for m in "$@"; do
  (mkdir -p scratch/abl/o$m && for f in pycsou_amd/csrc/*.hip; do
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -DPCS_ABLATE=$m -c $f -o scratch/abl/o$m/$(basename $f .hip).o || exit 1
   done && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scratch/abl/lib$m.so scratch/abl/o$m/*.o) &
done
wait
