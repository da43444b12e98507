#!/bin/bash
# Same-box A/B of library builds: tools/ab.sh TAG LIB_A LIB_B [ROUNDS]
# Alternates `bench.py` runs with TMH_LIB pointing at each build (ABAB...),
# one JSON line per run in gpurun_out/ab_TAG.jsonl.  Box-to-box spread of the
# same build is several percent, so compare only within one call.
set -u
TAG=$1; A=$2; B=$3; R=${4:-3}
mkdir -p gpurun_out
: > gpurun_out/ab_$TAG.jsonl
for i in $(seq 1 $R); do
  for L in $A $B; do
    TMH_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras \
      > gpurun_out/ab_$TAG.tmp 2>> gpurun_out/ab_$TAG.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$TAG.tmp')); print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $L >> gpurun_out/ab_$TAG.jsonl
    tail -1 gpurun_out/ab_$TAG.jsonl
  done
done
