#!/bin/bash
# Build libtmhip.so (and libtmh5.so) on the GPU box from the pushed sources
# (csrc/build is not pushed, so every object is recompiled), logging the
# toolchain: the GPU tests and bench then run the library built from HEAD.
set -u
mkdir -p gpurun_out
TAG=${1:-run}
L=gpurun_out/build_$TAG.log
{ /opt/rocm/bin/hipcc --version; echo; } > $L 2>&1
timeout -k 10 120 make -C tmlibrary_amd/csrc clean >> $L 2>&1 || exit $?
timeout -k 10 900 make -C tmlibrary_amd/csrc -j16 >> $L 2>&1 || exit $?
if [ -f /opt/conda/include/hdf5.h ]; then timeout -k 10 300 make -C tmlibrary_amd/csrc h5 >> $L 2>&1 || exit $?; fi
sha256sum tmlibrary_amd/hip/*.so >> $L
echo build-ok >> $L
