#!/bin/bash
# r3t: host-streamed configs[4] vs the HIP hardware-queue count (false stream dependencies)
mkdir -p gpurun_out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python3 bench.py --stream-host --stream-channels 3 --stream-sites 4096 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/stream_host_q${q}_r3t.json 2> gpurun_out/stream_host_q${q}_r3t.err || exit $?
done
