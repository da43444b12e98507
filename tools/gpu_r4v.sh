#!/bin/bash
# r4v: code lengths aliased into lfast, 16-dword ring (10 workgroups per CU)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4v || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4v.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4v.log; tail -3 gpurun_out/gpu_tests_inflate_r4v.log
if [ $rc -ne 0 ]; then exit $rc; fi
TMH_LIB=build_ab/zprof1/libtmhip.so timeout -k 10 400 python tools/inflate_prof.py --block 128 --lanes 8 > gpurun_out/zprof_r4v.json 2> gpurun_out/zprof_r4v.err || exit $?
cat gpurun_out/zprof_r4v.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16 > gpurun_out/bench_inflate_r4v.json 2> gpurun_out/bench_inflate_r4v.err || exit $?
cat gpurun_out/bench_inflate_r4v.json
timeout -k 10 500 python tools/bench_input_path.py --blocks 128 > gpurun_out/input_path_r4v.jsonl 2> gpurun_out/input_path_r4v.err || exit $?
cat gpurun_out/input_path_r4v.jsonl
TMH_LIB=build_ab/ring32/libtmhip.so timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 > gpurun_out/bench_inflate_ring32_r4v.json 2> gpurun_out/bench_inflate_ring32_r4v.err || exit $?
cat gpurun_out/bench_inflate_ring32_r4v.json
echo r4v-ok
