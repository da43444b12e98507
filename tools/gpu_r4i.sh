#!/bin/bash
# r4i: inflate phase 1 with global-address-space output stores; lanes sweep
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4i || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4i.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4i.log; tail -3 gpurun_out/gpu_tests_inflate_r4i.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16,32,64 > gpurun_out/bench_inflate_r4i.json 2> gpurun_out/bench_inflate_r4i.err || exit $?
cat gpurun_out/bench_inflate_r4i.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 384 --reps 2 --lanes 8,16,32 > gpurun_out/bench_inflate_b384_r4i.json 2> gpurun_out/bench_inflate_b384_r4i.err || exit $?
cat gpurun_out/bench_inflate_b384_r4i.json
echo r4i-ok
