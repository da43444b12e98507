#!/bin/bash
# r4b: in-pass finalize without agent-scope fences: epochs A/B (standard and
# bright), forced-distributed 4-channel run with every channel checked
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4b || exit $?
ab() {  # ab TAG EXTRA-ARGS EPOCHS...
  local tag=$1 extra=$2; shift 2
  for E in "$@"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --fused-epochs $E $extra > gpurun_out/ab_e.tmp 2>> gpurun_out/ab_$tag.err || return $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_e.tmp').read().strip().splitlines()[-1]); print(json.dumps({'epochs': int(sys.argv[1]), 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $E >> gpurun_out/ab_$tag.jsonl
    tail -1 gpurun_out/ab_$tag.jsonl
  done
}
ab epochs_r4b "" 0 4 1 8 2 16 0 4 || exit $?
ab epochs_bright_r4b "--distribution bright" 0 4 8 0 4 || exit $?
TMH_BENCH_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --layout sharded --channels 4 --sites 3456 --steps 3 --warmup 1 --no-extras --cpu-sample 0 > gpurun_out/dist4_r4b.json 2> gpurun_out/dist4_r4b.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/dist4_r4b.json')); print(d['value'], d['ms_per_step'], d['check_vs_oracle'], d['check'].get('channels_checked'))"
echo r4b-ok
