#!/bin/bash
# r3d: Welford code-vs-placement check, fold tail timing, bench x2, input path thread scaling
mkdir -p gpurun_out
timeout -k 10 200 ./tools/mb/mb_place2 3456 2 2 64 > gpurun_out/mb_place2_r3d.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3d.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_r3d.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/bench_r3d_$i.json 2> gpurun_out/bench_r3d_$i.err || exit $?; done
for t in 16 32 64 128; do timeout -k 10 300 python tools/bench_input.py --sites 64 --threads $t --no-gpu > gpurun_out/input_r3d_$t.json 2> gpurun_out/input_r3d_$t.err || exit $?; done
