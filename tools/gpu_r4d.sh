#!/bin/bash
# r4d: can one launch shape serve both standard and bright sites?  Welford in
# the bright shape (1,024 threads, 16,384-entry LUT) on standard sites; the
# packed fused configuration (5) on standard sites.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_multi.sh wf1k_std_r4d 2 tmlibrary_amd/hip/libtmhip.so build_ab/wf1k/libtmhip.so || exit $?
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh wf1k_bright_r4d 1 tmlibrary_amd/hip/libtmhip.so build_ab/wf1k/libtmhip.so || exit $?
BENCH_ARGS="--fused-config 5" bash tools/ab_multi.sh cfg5_std_r4d 1 tmlibrary_amd/hip/libtmhip.so || exit $?
BENCH_ARGS="--fused-config 3" bash tools/ab_multi.sh cfg3_std_r4d 1 tmlibrary_amd/hip/libtmhip.so || exit $?
BENCH_ARGS="--fused-config 5" bash tools/ab_multi.sh cfg5b_std_r4d 1 tmlibrary_amd/hip/libtmhip.so || exit $?
echo r4d-ok
