#!/bin/bash
# r4f: GPU inflate -- parity tests, then the input-path throughput
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4f || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4f.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4f.log
tail -15 gpurun_out/gpu_tests_inflate_r4f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 > gpurun_out/bench_inflate_r4f.json 2> gpurun_out/bench_inflate_r4f.err || exit $?
cat gpurun_out/bench_inflate_r4f.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k run_job -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_runjob_r4f.log 2>&1 || exit $?
timeout -k 10 900 python tools/bench_input.py --sites 64 --threads 16 --repeat 4 > gpurun_out/bench_input_r4f.json 2> gpurun_out/bench_input_r4f.err || exit $?
cat gpurun_out/bench_input_r4f.json
echo r4f-ok
