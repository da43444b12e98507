#!/bin/bash
# r3z4: chain pass flag rule (group bound vs launch-wide T, fix-kernel recheck): tests, mb, bench chain stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3z4.log 2>&1 || exit $?
timeout -k 10 400 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3z4.txt 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3z4 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/prof_r3z4.log 2>&1 || exit $?
