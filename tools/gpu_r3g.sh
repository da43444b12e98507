#!/bin/bash
# r3g: Welford 3-stage pipeline + block cursor; dense tail default; fold2 as the fold option
mkdir -p gpurun_out
timeout -k 10 200 ./tools/mb/mb_place2 3456 2 2 64 > gpurun_out/mb_place2_r3g.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3g.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r3g.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/bench_r3g_$i.json 2> gpurun_out/bench_r3g_$i.err || exit $?; done
