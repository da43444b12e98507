#!/bin/bash
# r3z12: kernel trace of the N=8 shard size (4 channels x 432 sites) on one rank, forced distributed path
mkdir -p gpurun_out
export TMPDIR=/tmp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 TMH_BENCH_FORCE_DIST=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3z12 -o run -- python3 bench.py --layout sharded --channels 4 --sites 432 --steps 5 --warmup 2 --no-extras --cpu-sample 0 > gpurun_out/prof_r3z12.log 2>&1 || exit $?
