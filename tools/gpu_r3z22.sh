#!/bin/bash
# r3z22: bright Welford pass -- ablation without the >= 16,384 rare path (wrong statistics; timing only)
mkdir -p gpurun_out
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh wfr 2 build_ab/wfr_base/libtmhip.so build_ab/wfr_abl/libtmhip.so || exit $?
