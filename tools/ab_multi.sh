#!/bin/bash
# Same-box A/B/C/... of library builds: tools/ab_multi.sh TAG ROUNDS LIB...
# bench.py runs with TMH_LIB pointing at each build, the order reversed every
# other round (A B B A ...): successive bench processes on one box drift
# (profiles/r2/drift_same_lib_r2zb.jsonl: the same build 13.22 -> 14.69 ms
# for correct_hist over five runs), so a fixed order would favour the first
# build.  One JSON line per run in gpurun_out/ab_TAG.jsonl; compare only
# within one call.
set -u
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
: > gpurun_out/ab_$TAG.jsonl
LIBS=("$@")
for i in $(seq 1 $R); do
  ORDER=("${LIBS[@]}")
  if [ $((i % 2)) -eq 0 ]; then
    ORDER=(); for ((j=${#LIBS[@]}-1; j>=0; j--)); do ORDER+=("${LIBS[j]}"); done
  fi
  for L in "${ORDER[@]}"; do
    TMH_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras ${BENCH_ARGS:-} \
      > gpurun_out/ab_$TAG.tmp 2>> gpurun_out/ab_$TAG.err || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$TAG.tmp') if l.strip()][-1]); print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $L >> gpurun_out/ab_$TAG.jsonl
    tail -1 gpurun_out/ab_$TAG.jsonl
  done
done
