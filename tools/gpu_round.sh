#!/bin/bash
# tests -> smoke -> bench -> rocprofv3 kernel trace.  Every GPU step has its
# own time limit; a crash/abort/timeout (rc other than 0/1 for pytest, other
# than 0 for the rest) ends the script there.
set -u
TAG=${1:-run}
STEPS=${STEPS:-5}
CPUS=${CPUS:-24}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps $STEPS --warmup 2 --cpu-sample $CPUS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/prof_$TAG.log 2>&1 || exit $?
find gpurun_out/prof_$TAG -name "*stats*" | head
