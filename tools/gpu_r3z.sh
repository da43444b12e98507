#!/bin/bash
# r3z: the new chain overflow test, full GPU suite + smoke, bench with extras (chain)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain_r3z.log 2>&1 || exit $?
bash tools/gpu_check.sh r3z || exit $?
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r3z.json 2> gpurun_out/bench_r3z.err || exit $?
