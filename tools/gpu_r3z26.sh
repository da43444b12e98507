#!/bin/bash
# r3z26: bright Welford rare path all eight slots computed then selected inside the thread branch: blocked/bright parity tests, bright A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocked.py tests/test_gpu_fullsize.py -x -q -k "bright or blocked" --timeout 300 --timeout-method thread > gpurun_out/pytest_wfr_r3z26.log 2>&1 || exit $?
BENCH_ARGS="--distribution bright" bash tools/ab_multi.sh wfr4 2 build_ab/wfr_base/libtmhip.so build_ab/wfr_new/libtmhip.so || exit $?
