#!/bin/bash
# r3z19: first-allocation placement: 0 / 40 / 80 GB held before the site buffers, order reversed every other round
mkdir -p gpurun_out
: > gpurun_out/hbm_skip_r3z19.jsonl
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then L="0 40 80"; else L="80 40 0"; fi
  for g in $L; do
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --hbm-skip-gb $g > gpurun_out/hbm_skip_tmp.json 2>> gpurun_out/hbm_skip_r3z19.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/hbm_skip_tmp.json') if l.startswith('{')][-1]); print(json.dumps({'skip_gb': $g, 'value': d['value'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items() if k in ('welford', 'correct_hist')}}))" >> gpurun_out/hbm_skip_r3z19.jsonl
  done
done
