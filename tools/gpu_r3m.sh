#!/bin/bash
# r3m: bright Welford pass (16K exact LUT, 1024-thread workgroups) -- tests, bright + standard A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3m.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r3m.log
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh wfb_bright_r3m 2 build_ab/wfb_old/libtmhip.so build_ab/wfb_new/libtmhip.so || exit $?
bash tools/ab_multi.sh wfb_std_r3m 1 build_ab/wfb_old/libtmhip.so build_ab/wfb_new/libtmhip.so
