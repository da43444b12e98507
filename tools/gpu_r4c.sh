#!/bin/bash
# r4c: distributed layout at the N=8 shard size (4 channels x 432 sites, one
# rank, forced-distributed): fused-pass grid size and stream layout A/B, and a
# kernel trace of the default for the timeline
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_build.sh r4c || exit $?
: > gpurun_out/dist432_r4c.jsonl
run() {  # run TAG ARGS...
  local tag=$1; shift
  TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
    timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 --warmup 3 \
    --no-extras --cpu-sample 0 "$@" > gpurun_out/d.tmp 2>> gpurun_out/dist432_r4c.err || return $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/d.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $tag >> gpurun_out/dist432_r4c.jsonl
  tail -1 gpurun_out/dist432_r4c.jsonl
}
run default || exit $?
run cus224 --fused-cus 224 || exit $?
run cus192 --fused-cus 192 || exit $?
run cus160 --fused-cus 160 || exit $?
run onestream --channel-streams one || exit $?
run default || exit $?
run cus192 --fused-cus 192 || exit $?
TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29518 \
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace432_r4c -o run -- \
  python3 bench.py --layout sharded --channels 4 --sites 432 --steps 3 --warmup 1 --no-extras --cpu-sample 0 --no-profile \
  > gpurun_out/trace432_r4c.log 2>&1 || exit $?
echo r4c-ok
