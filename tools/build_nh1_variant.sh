#!/bin/bash
# Fast A/B variant of the library: only the NH=1 translation unit (bw <= 63)
# is recompiled with the given flags; every other object comes from the
# in-tree build (build/obj_libunipeak_hip, run tools/build.py first).
# usage: tools/build_nh1_variant.sh NAME -DFLAG ...  -> unipeak_amd/lib/libunipeak_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
N=$1; shift
O=build/obj_libunipeak_hip; V=build/obj_nh1_$N; mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I include \
  -DUPK_NH_TU=1 "$@" -c -o $V/nh1.o unipeak_amd/csrc/nh_tu.hip
objs=$(ls $O/*.o | grep -v '/nh1.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o unipeak_amd/lib/libunipeak_hip_$N.so $objs $V/nh1.o
echo built unipeak_amd/lib/libunipeak_hip_$N.so
