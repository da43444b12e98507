#!/bin/bash
# r3z18: first-allocation placement: bench with 0 / 40 GB held before the site buffers, alternating processes
mkdir -p gpurun_out
: > gpurun_out/hbm_skip_r3z18.jsonl
for i in 1 2 3; do
  for g in 0 40; do
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --hbm-skip-gb $g > gpurun_out/hbm_skip_tmp.json 2>> gpurun_out/hbm_skip_r3z18.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/hbm_skip_tmp.json') if l.startswith('{')][-1]); print(json.dumps({'skip_gb': $g, 'value': d['value'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items() if k in ('welford', 'correct_hist')}}))" >> gpurun_out/hbm_skip_r3z18.jsonl
  done
done
