#!/bin/bash
# Build a diagnostic variant of the engine: tools/build_var.sh NAME -DFLAG=... ; the library lands in
# pycsou_amd/lib/var/NAME/libpycsou_hip.so (select it with PCS_LIB_PATH).  VAR_ONLY="sep_ata pds" compiles
# only those sources with the flags and links the in-tree build's objects (build/*.o, `make` first) for the rest.
cd "$(dirname "$0")/.." || exit 1
name=$1; shift
o=build/var_$name; rm -rf $o; mkdir -p $o pycsou_amd/lib/var/$name
pids=()
for f in pycsou_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ -n "$VAR_ONLY" ] && ! [[ " $VAR_ONLY " == *" $b "* ]]; then
    cp build/$b.o $o/$b.o || exit 1
    continue
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -fPIC -std=c++17 -Iinclude "$@" -c $f -o $o/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || exit 1; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o pycsou_amd/lib/var/$name/libpycsou_hip.so $o/*.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
