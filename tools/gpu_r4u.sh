#!/bin/bash
# r4u: inflate data loop with 32-bit counters, consumed bits from the ring position
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4u || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4u.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4u.log; tail -3 gpurun_out/gpu_tests_inflate_r4u.log
if [ $rc -ne 0 ]; then exit $rc; fi
TMH_LIB=build_ab/zprof1/libtmhip.so timeout -k 10 400 python tools/inflate_prof.py --block 128 --lanes 8 > gpurun_out/zprof_r4u.json 2> gpurun_out/zprof_r4u.err || exit $?
cat gpurun_out/zprof_r4u.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16 > gpurun_out/bench_inflate_r4u.json 2> gpurun_out/bench_inflate_r4u.err || exit $?
cat gpurun_out/bench_inflate_r4u.json
timeout -k 10 500 python tools/bench_input_path.py --blocks 128 > gpurun_out/input_path_r4u.jsonl 2> gpurun_out/input_path_r4u.err || exit $?
cat gpurun_out/input_path_r4u.jsonl
echo r4u-ok
