#!/bin/bash
# r3o: blocked ordered sum (k_pct_acc_blk), fixups beside the tail, 4,096-group probe
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3o.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r3o.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 ./tools/mb/mb_fold 3456 5 0 > gpurun_out/mb_fold_r3o.txt 2>&1 || exit $?
bash tools/ab_multi.sh tail_r3o 3 build_ab/tail_old/libtmhip.so build_ab/tail_new/libtmhip.so
