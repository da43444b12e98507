#!/bin/bash
# Build an A/B variant of libtmhip.so from the sources in build_ab/NAME
# (a copy of tmlibrary_amd/csrc with some files swapped):
#   tools/build_variant.sh NAME   ->  build_ab/NAME/libtmhip.so
set -eu
D=build_ab/$1
mkdir -p $D/include $D/obj
cp include/tmhip.h $D/include/
for f in abi stats_kernels apply_kernels fused_kernels chain_kernels synth_kernels inflate_kernels; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas --offload-arch=gfx950 \
    -I$D/include -I$D -c $D/$f.hip -o $D/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $D/libtmhip.so $D/obj/*.o
