#!/bin/bash
# r3n: chain pass with two-stage buffer loads (old vs new, checksums)
mkdir -p gpurun_out
timeout -k 10 300 ./tools/mb/mb_chain_old 3456 3 > gpurun_out/mb_chain_old_r3n.txt 2>&1 || exit $?
timeout -k 10 300 ./tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_new_r3n.txt 2>&1 || exit $?
timeout -k 10 300 ./tools/mb/mb_chain_old 3456 3 > gpurun_out/mb_chain_old2_r3n.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_chain_r3n.log 2>&1
