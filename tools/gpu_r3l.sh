#!/bin/bash
# r3l: input path thread scaling (decode only, then one run_job line), granted cores
mkdir -p gpurun_out
for t in 8 16 32 64 128; do
  timeout -k 10 300 python tools/bench_input.py --sites 128 --threads $t --no-gpu > gpurun_out/input_r3l_$t.json 2> gpurun_out/input_r3l_$t.err || exit $?
done
timeout -k 10 400 python tools/bench_input.py --sites 128 --threads 16 > gpurun_out/input_r3l_gpu16.json 2> gpurun_out/input_r3l_gpu16.err || exit $?
