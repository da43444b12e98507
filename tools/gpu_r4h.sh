#!/bin/bash
# r4h: GPU inflate with buffered 16-byte output stores, paired match-list
# stores, 2-deep bit-buffer prefetch and a lanes-per-workgroup sweep; run_job
# with GPU decode; the full GPU suite; the headline bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4h || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_inflate_r4h.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_inflate_r4h.log; tail -16 gpurun_out/gpu_tests_inflate_r4h.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16,32,64 > gpurun_out/bench_inflate_r4h.json 2> gpurun_out/bench_inflate_r4h.err || exit $?
cat gpurun_out/bench_inflate_r4h.json
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 384 --reps 2 --lanes 8,16 > gpurun_out/bench_inflate_b384_r4h.json 2> gpurun_out/bench_inflate_b384_r4h.err || exit $?
cat gpurun_out/bench_inflate_b384_r4h.json
timeout -k 10 900 python tools/bench_input.py --sites 64 --threads 16 --repeat 4 > gpurun_out/bench_input_r4h.json 2> gpurun_out/bench_input_r4h.err || exit $?
cat gpurun_out/bench_input_r4h.json
bash tools/gpu_check.sh r4h
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_r4h.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r4h.json 2> gpurun_out/bench_r4h.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_r4h.json')); print(d['value'], d['check_vs_oracle'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d['extras'].get('input_path'))"
echo r4h-ok
