#!/bin/bash
# build a variant of the HIP library: tools/build_variant.sh NAME -DFLAG ...
# -> unipeak_amd/lib/libunipeak_hip_NAME.so (load with UNIPEAK_LIB=...)
cd "$(dirname "$0")/.." || exit 1
name=$1; shift
exec /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -I include "$@" -o "unipeak_amd/lib/libunipeak_hip_$name.so" unipeak_amd/csrc/api.hip
