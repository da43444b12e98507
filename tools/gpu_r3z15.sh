#!/bin/bash
# r3z15: histogram finalize at 512 threads per site (2-round super-rounds) vs 1,024 (4-round): same-box A/B, standard and bright
mkdir -p gpurun_out
bash tools/ab_multi.sh fin 3 build_ab/fin_old/libtmhip.so build_ab/fin_new/libtmhip.so || exit $?
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh finb 2 build_ab/fin_old/libtmhip.so build_ab/fin_new/libtmhip.so || exit $?
