#!/bin/bash
# microbenchmarks + bench (+ optional rocprof), each GPU step time-limited;
# stops at the first crash/timeout.
set -u
TAG=${1:-perf}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/mb/mb_stats ]; then
  timeout -k 10 300 tools/mb/mb_stats ${MB_SITES:-1024} 3 > gpurun_out/mb_$TAG.txt 2>&1 || exit $?
fi
timeout -k 10 900 python bench.py --steps ${STEPS:-5} --warmup 2 --cpu-sample ${CPUS:-0} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/prof_$TAG.log 2>&1 || exit $?
fi
echo ok
