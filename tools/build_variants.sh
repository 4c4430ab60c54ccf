#!/bin/bash
# tools/build_variants.sh NAME="-DFLAG ..." ... — builds experiment variants of libhippt.so as
# qt-raytracer_amd/libv_NAME.so (git-ignored; they travel to the GPU box) for A/B runs with
# HIPPT_LIB=qt-raytracer_amd/libv_NAME.so.  Same flags as the Makefile plus the given defines.
set -euo pipefail
cd "$(dirname "$0")/../qt-raytracer_amd"
SRC="csrc/hippt_kernels.hip csrc/hippt_wavefront.hip csrc/hippt_api.cpp csrc/bvh_builder.cpp csrc/item_order.cpp csrc/mesh_io.cpp"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -shared -Wl,--version-script=csrc/exports.map"
for spec in "$@"; do
    name=${spec%%=*}
    defs=${spec#*=}
    /opt/rocm/bin/hipcc $FLAGS $defs -o libv_$name.so $SRC &
done
wait
ls -la libv_*.so
