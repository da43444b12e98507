#!/bin/bash
# r3z9: chain fix kernel one thread per pixel: chain tests, kernel stats of a bench run with extras
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3z9.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3z9 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/prof_r3z9.log 2>&1 || exit $?
