#!/bin/bash
# r4n: inflate data path as its own loop (branch-free ring refills)
# flight across iterations); counters; lanes sweep at 128 and 384 sites
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4n || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4n.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4n.log; tail -3 gpurun_out/gpu_tests_inflate_r4n.log
if [ $rc -ne 0 ]; then exit $rc; fi
TMH_LIB=build_ab/zprof1/libtmhip.so timeout -k 10 400 python tools/inflate_prof.py --block 128 --lanes 8,64 > gpurun_out/zprof_r4n.json 2> gpurun_out/zprof_r4n.err || exit $?
cat gpurun_out/zprof_r4n.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16,32,64 > gpurun_out/bench_inflate_r4n.json 2> gpurun_out/bench_inflate_r4n.err || exit $?
cat gpurun_out/bench_inflate_r4n.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 384 --reps 2 --lanes 8,16,32 > gpurun_out/bench_inflate_b384_r4n.json 2> gpurun_out/bench_inflate_b384_r4n.err || exit $?
cat gpurun_out/bench_inflate_b384_r4n.json
echo r4n-ok
