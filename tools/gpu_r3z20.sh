#!/bin/bash
# r3z20: fused configuration 5 (packed u16 counters, 4 sites x 16,384 bins, 8 bands): parity tests, bright A/B vs configuration 0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -k "packed or multi_job or very_wide" --timeout 300 --timeout-method thread > gpurun_out/pytest_pk_r3z20.log 2>&1 || exit $?
: > gpurun_out/pk_ab_r3z20.jsonl
for i in 1 2; do
  if [ $i -eq 1 ]; then L="0 5"; else L="5 0"; fi
  for c in $L; do
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --distribution bright --fused-config $c > gpurun_out/pk_tmp.json 2>> gpurun_out/pk_ab_r3z20.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pk_tmp.json') if l.startswith('{')][-1]); print(json.dumps({'cfg': $c, 'value': d['value'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" >> gpurun_out/pk_ab_r3z20.jsonl
  done
done
