#!/bin/bash
# Successive bench processes on one box: is the fused pass's drift thermal
# (gone with pauses between runs) or allocation state (stays)?
# usage: tools/drift_probe.sh TAG RUNS PAUSE_S
set -u
TAG=$1; R=$2; P=$3
mkdir -p gpurun_out
: > gpurun_out/drift_$TAG.jsonl
for i in $(seq 1 $R); do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras \
    > gpurun_out/drift_$TAG.tmp 2>> gpurun_out/drift_$TAG.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/drift_$TAG.tmp')); print(json.dumps({'run': int(sys.argv[1]), 'pause_s': int(sys.argv[2]), 'value': d['value'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $i $P >> gpurun_out/drift_$TAG.jsonl
  tail -1 gpurun_out/drift_$TAG.jsonl
  sleep $P
done
