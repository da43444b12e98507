#!/bin/bash
# r3q: Welford at five workgroups per CU (96 VGPRs, 32 KB LDS) vs four
mkdir -p gpurun_out
timeout -k 10 300 ./tools/mb/mb_welford_old 3456 3 0 > gpurun_out/mb_welford_old_r3q.txt 2>&1 || exit $?
timeout -k 10 300 ./tools/mb/mb_welford 3456 3 0 > gpurun_out/mb_welford_new_r3q.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_blocked.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3q.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_r3q.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_multi.sh wf5_r3q 3 build_ab/wf5_oldlib/libtmhip.so build_ab/wf5_new/libtmhip.so
