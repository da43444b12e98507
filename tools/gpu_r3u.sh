#!/bin/bash
# r3u: configs[2] code path (4 channels on 4 streams, forced distributed, one rank) vs HW queue count
mkdir -p gpurun_out
p=29517
for q in 4 8 16 4; do
  p=$((p+1))
  GPU_MAX_HW_QUEUES=$q TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --layout sharded --channels 4 --sites 864 --steps 5 --warmup 2 --no-extras --cpu-sample 0 > gpurun_out/dist4_q${q}_${p}_r3u.json 2> gpurun_out/dist4_q${q}_${p}_r3u.err || exit $?
done
