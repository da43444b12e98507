#!/bin/bash
# r3z11: configs[2] per-GPU shard sizes on one rank (forced distributed path, 4 channels):
# 432 sites/channel = the N=8 shard, 864 = N=4, 1728 = N=2
mkdir -p gpurun_out
p=29600
: > gpurun_out/dist4_shards_r3z11.jsonl
for n in 432 864 1728; do
  p=$((p+1))
  TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --layout sharded --channels 4 --sites $n --steps 5 --warmup 2 --no-extras --cpu-sample 0 >> gpurun_out/dist4_shards_r3z11.jsonl 2> gpurun_out/dist4_shards_${n}_r3z11.err || exit $?
done
