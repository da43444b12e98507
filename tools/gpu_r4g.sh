#!/bin/bash
# r4g: GPU inflate (tests, kernel A/B: first-level tables vs canonical search
# only), run_job with GPU decode, then the full GPU suite and the headline bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4g || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4g.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4g.log; tail -14 gpurun_out/gpu_tests_inflate_r4g.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 > gpurun_out/bench_inflate_r4g.json 2> gpurun_out/bench_inflate_r4g.err || exit $?
cat gpurun_out/bench_inflate_r4g.json
TMH_LIB=build_ab/inflate_base/libtmhip.so timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 > gpurun_out/bench_inflate_base_r4g.json 2> gpurun_out/bench_inflate_base_r4g.err || exit $?
cat gpurun_out/bench_inflate_base_r4g.json
timeout -k 10 900 python tools/bench_input.py --sites 64 --threads 16 --repeat 4 > gpurun_out/bench_input_r4g.json 2> gpurun_out/bench_input_r4g.err || exit $?
cat gpurun_out/bench_input_r4g.json
bash tools/gpu_check.sh r4g
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_r4g.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r4g.json 2> gpurun_out/bench_r4g.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r4g.json')); print(d['value'], d['check_vs_oracle'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d['extras'].get('input_path'))"
echo r4g-ok
