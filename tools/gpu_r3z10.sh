#!/bin/bash
# r3z10: fused-pass f64 fixups one thread per pixel: GPU suite + smoke, kernel stats, two bench runs
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh r3z10 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3z10 -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras > gpurun_out/prof_r3z10.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/bench_r3z10_$i.json 2> gpurun_out/bench_r3z10_$i.err || exit $?
done
