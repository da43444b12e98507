#!/bin/bash
# Same-box A/B of bench.py argument sets: tools/ab_args.sh TAG ROUNDS "ARGS_A" "ARGS_B" ...
# Runs every argument set once per round (round-robin), one JSON line per run
# in gpurun_out/ab_TAG.jsonl.
set -u
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
: > gpurun_out/ab_$TAG.jsonl
for i in $(seq 1 $R); do
  for ARGS in "$@"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras $ARGS \
      > gpurun_out/ab_$TAG.tmp 2>> gpurun_out/ab_$TAG.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$TAG.tmp')); print(json.dumps({'args': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" "$ARGS" >> gpurun_out/ab_$TAG.jsonl
    tail -1 gpurun_out/ab_$TAG.jsonl
  done
done
