#!/bin/bash
# build a variant of the HIP library: tools/build_variant.sh NAME -DFLAG ...
# -> unipeak_amd/lib/libunipeak_hip_NAME.so (load with UNIPEAK_LIB=...)
cd "$(dirname "$0")/.." || exit 1
exec python3 tools/build.py --variant "$@"
