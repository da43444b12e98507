#!/bin/bash
# r3z21: packed configuration as the automatic wide choice: GPU suite + smoke; bright A/B 8 vs 4 bands
mkdir -p gpurun_out
bash tools/gpu_check.sh r3z21 || exit $?
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh pkb 2 build_ab/pk8/libtmhip.so build_ab/pk4/libtmhip.so || exit $?
