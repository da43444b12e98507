#!/bin/bash
# r3s: configs[4] host-streamed run, uniform-distribution job, on the current build
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --stream-host --stream-channels 3 --stream-sites 4096 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/stream_host_r3s.json 2> gpurun_out/stream_host_r3s.err || exit $?
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras --distribution uniform > gpurun_out/bench_uniform_r3s.json 2> gpurun_out/bench_uniform_r3s.err || exit $?
