#!/bin/bash
# tests + smoke -> bench (N=1, configs[1]) -> single-rank forced-distributed
# 4-channel sharded bench (configs[2] code path) -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout (rc other than
# 0/1 for pytest, other than 0 for the rest) ends the script there.
# SKIP_TESTS=1 skips the test step.
set -u
TAG=${1:-run}
STEPS=${STEPS:-10}
CPUS=${CPUS:-96}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  bash tools/gpu_check.sh $TAG
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 900 python bench.py --steps $STEPS --warmup 3 --cpu-sample $CPUS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
if [ "${SKIP_DIST:-0}" != "1" ]; then
  TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --layout sharded --channels 4 --sites 864 --steps 5 --warmup 2 --no-extras --cpu-sample 0 > gpurun_out/dist4_$TAG.json 2> gpurun_out/dist4_$TAG.err || exit $?
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras > gpurun_out/prof_$TAG.log 2>&1 || exit $?
fi
echo round-ok
