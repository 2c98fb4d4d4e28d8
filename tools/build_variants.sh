#!/bin/bash
# Build libacnerf.so variants (developer A/B tool).  Each argument is
#   name:source.hip:"-DFLAG=V -DFLAG2=V"   -> build_variants/libacnerf_<name>.so
# (the named source recompiled with the flags, every other object from the regular build)
set -e
cd "$(dirname "$0")/../adaptive_city_nerf_amd/csrc"
make -s >/dev/null
mkdir -p ../../build_variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; defs=${rest#*:}
  objs=""
  for o in build/*.o; do
    [ "$o" = "build/$src.o" ] || objs="$objs $o"
  done
  ( /opt/rocm/bin/hipcc $F $defs -c $src -o /tmp/${src%.hip}_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build_variants/libacnerf_$name.so \
      $objs /tmp/${src%.hip}_$name.o && echo "built $name" ) &
done
wait
