#!/bin/bash
# r3w: trimmed chain pass (k_chain_u8t) -- microbenchmark (checksums vs the
# previous form) and the chain GPU parity tests
mkdir -p gpurun_out
timeout -k 10 300 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3w.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3w.log 2>&1 || exit $?
