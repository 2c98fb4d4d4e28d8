#!/bin/bash
# Build libacnerf.so variants of render.hip (developer A/B tool).  Each argument is
#   name:"-DFLAG=V -DFLAG2=V"   -> build_variants/libacnerf_<name>.so
set -e
cd "$(dirname "$0")/../adaptive_city_nerf_amd/csrc"
make -s >/dev/null
mkdir -p ../../build_variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  ( /opt/rocm/bin/hipcc $F $defs -c render.hip -o /tmp/render_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build_variants/libacnerf_$name.so \
      build/capi_common.cpp.o build/encoders.hip.o build/rays.hip.o build/optim.hip.o /tmp/render_$name.o && echo "built $name" ) &
done
wait
