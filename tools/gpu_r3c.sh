#!/bin/bash
# r3c: blocked Welford/fused microbenchmark, GPU tests (fold tail), two bench runs
mkdir -p gpurun_out
timeout -k 10 200 ./tools/mb/mb_place2 3456 2 2 64,16 > gpurun_out/mb_place2_r3c.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3c.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r3c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/bench_r3c_$i.json 2> gpurun_out/bench_r3c_$i.err || exit $?; done
