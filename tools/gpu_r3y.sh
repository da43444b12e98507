#!/bin/bash
# r3y: chain pass -- 32-bit staging arithmetic, part counts, unshifted ablation; chain tests
mkdir -p gpurun_out
timeout -k 10 400 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3y.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3y.log 2>&1 || exit $?
