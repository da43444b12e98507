#!/bin/bash
# r3z13: 4 channels on one rank (forced distributed path): per-channel streams vs one stream, N=8 and N=4 shard sizes
mkdir -p gpurun_out
p=29620
: > gpurun_out/dist4_streams_r3z13.jsonl
for n in 432 864; do
  for m in per-channel one per-channel one; do
    p=$((p+1))
    TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --layout sharded --channels 4 --sites $n --channel-streams $m --steps 5 --warmup 2 --no-extras --cpu-sample 0 --no-profile > gpurun_out/dist4_streams_tmp.json 2>> gpurun_out/dist4_streams_r3z13.err || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/dist4_streams_tmp.json') if l.startswith('{')][-1]); print(json.dumps({'sites': $n, 'streams': '$m', 'value': d['value'], 'ms': d['ms_per_step'], 'check': d.get('check_vs_oracle')}))" >> gpurun_out/dist4_streams_r3z13.jsonl
  done
done
