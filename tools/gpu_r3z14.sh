#!/bin/bash
# r3z14: k_pct_acc with two alternating register sets (precise waits): full-size parity tests, same-box A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full_r3z14.log 2>&1 || exit $?
bash tools/ab_multi.sh pct 3 build_ab/pct_old/libtmhip.so build_ab/pct_new/libtmhip.so || exit $?
