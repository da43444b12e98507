#!/bin/bash
# r4o: h5py's 135x160 chunks (the reference's layout), data loop without
# LDS code tables, H2D on its own stream; run_job with GPU decode; full suite
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4o || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4o.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4o.log; tail -3 gpurun_out/gpu_tests_inflate_r4o.log
if [ $rc -ne 0 ]; then exit $rc; fi
TMH_LIB=build_ab/zprof1/libtmhip.so timeout -k 10 400 python tools/inflate_prof.py --block 128 --lanes 8 > gpurun_out/zprof_r4o.json 2> gpurun_out/zprof_r4o.err || exit $?
cat gpurun_out/zprof_r4o.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16 > gpurun_out/bench_inflate_r4o.json 2> gpurun_out/bench_inflate_r4o.err || exit $?
cat gpurun_out/bench_inflate_r4o.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 256 --reps 2 --lanes 4,8 > gpurun_out/bench_inflate_b256_r4o.json 2> gpurun_out/bench_inflate_b256_r4o.err || exit $?
cat gpurun_out/bench_inflate_b256_r4o.json
timeout -k 10 900 python tools/bench_input.py --sites 128 --threads 16 --repeat 6 --device-block 128 > gpurun_out/bench_input_r4o.json 2> gpurun_out/bench_input_r4o.err || exit $?
cat gpurun_out/bench_input_r4o.json
bash tools/gpu_check.sh r4o
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_r4o.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r4o.json 2> gpurun_out/bench_r4o.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r4o.json')); print(d['value'], d['check_vs_oracle'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d['extras'].get('input_path'))"
echo r4o-ok
