#!/bin/bash
# r3i: input layout A/B (contiguous input + blocked output vs both blocked), same box
mkdir -p gpurun_out
: > gpurun_out/ab_inlayout_r3i.jsonl
for i in 1 2 3; do
  for L in contiguous blocked; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --in-layout $L > gpurun_out/r3i.tmp 2>> gpurun_out/r3i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r3i.tmp').read().strip().splitlines()[-1]); print(json.dumps({'in_layout': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $L >> gpurun_out/ab_inlayout_r3i.jsonl
  done
done
