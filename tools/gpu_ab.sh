#!/bin/bash
# A/B bench variants on one box: each argument is "TAG|ENV=.. ENV=..|bench args".
# Each run is time-limited; the script stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  echo "== $tag: $envs :: $args"
  env $envs timeout -k 10 400 python bench.py --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 $args \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "FAILED $tag rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
echo ok
