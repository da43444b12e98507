#!/bin/bash
# Round-3 measurement set on one box: GPU tests + smoke, PMC traffic (separate
# FETCH/WRITE passes), rocprofv3 kernel-trace stats, six headline bench
# processes, a bright bench, the forced-distributed 4-channel run.
set -u
TAG=${1:-r3f}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh $TAG
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile --no-extras"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 $B > gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 $B > gpurun_out/pmc_write_$TAG.log 2>&1 || { echo "write pass failed"; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG --sites 3456 --height 2160 --width 2560 -o profiles/pmc_traffic.json > gpurun_out/pmc_traffic_$TAG.log 2>&1 || { echo "pmc_traffic failed"; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras > gpurun_out/prof_$TAG.log 2>&1 || { echo "kernel trace failed"; exit 1; }
timeout -k 10 900 python3 bench.py --steps 10 --warmup 3 --cpu-sample 96 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; exit 1; }
: > gpurun_out/bench_repeat_$TAG.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras >> gpurun_out/bench_repeat_$TAG.jsonl 2>> gpurun_out/bench_repeat_$TAG.err || { echo "repeat $i failed"; exit 1; }
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --distribution bright > gpurun_out/bench_bright_$TAG.json 2> gpurun_out/bench_bright_$TAG.err || { echo "bright failed"; exit 1; }
TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --layout sharded --channels 4 --sites 864 --steps 5 --warmup 2 --no-extras --cpu-sample 0 > gpurun_out/dist4_$TAG.json 2> gpurun_out/dist4_$TAG.err || { echo "dist4 failed"; exit 1; }
echo final-ok
