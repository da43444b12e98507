#!/bin/bash
# r3j: fused pass with unconditional (out-of-bounds-safe) loads, ping-pong stages, LDS-staged fixups
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3j.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r3j.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_multi.sh fused_r3j 3 build_ab/fused_old/libtmhip.so build_ab/fused_new/libtmhip.so
