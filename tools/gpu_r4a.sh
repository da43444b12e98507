#!/bin/bash
# r4a: build on the box, GPU tests + smoke, default bench, in-pass finalize epochs A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4a || exit $?
bash tools/gpu_check.sh r4a
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || exit $?
: > gpurun_out/ab_epochs_r4a.jsonl
for E in 0 4 1 8 2 0 4; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --fused-epochs $E > gpurun_out/ab_e.tmp 2>> gpurun_out/ab_epochs_r4a.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_e.tmp').read().strip().splitlines()[-1]); print(json.dumps({'epochs': int(sys.argv[1]), 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $E >> gpurun_out/ab_epochs_r4a.jsonl
  tail -1 gpurun_out/ab_epochs_r4a.jsonl
done
echo r4a-ok
