#!/bin/bash
# Full measurement pass on a GPU box: PMC HBM traffic (separate FETCH/WRITE
# passes, kernel-trace only), rocprofv3 kernel-trace stats, then the bench
# line (which picks up the PMC traffic).  Every GPU step has its own time
# limit and the script stops at the first failure.
set -u
TAG=${1:-prof}
CPUS=${CPUS:-24}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 $B > gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo "fetch pass rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 $B > gpurun_out/pmc_write_$TAG.log 2>&1 || { echo "write pass rc=$?"; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG --sites 3456 --height 2160 --width 2560 -o profiles/pmc_traffic.json > gpurun_out/pmc_traffic_$TAG.log 2>&1 || { echo "pmc_traffic failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/prof_$TAG.log 2>&1 || { echo "kernel trace rc=$?"; exit 1; }
timeout -k 10 900 python3 bench.py --steps ${STEPS:-5} --warmup 2 --cpu-sample $CPUS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench rc=$?"; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$TAG.json
cat gpurun_out/bench_$TAG.json
echo ok
