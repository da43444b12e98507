#!/bin/bash
# r3z8: seam-line staging in production: chain tests, mb, bench (chain extra)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3z8.log 2>&1 || exit $?
timeout -k 10 500 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3z8.txt 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_r3z8.json 2> gpurun_out/bench_r3z8.err || exit $?
