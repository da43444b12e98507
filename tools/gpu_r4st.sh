#!/bin/bash
# r4st: the N = 8 shard-size layout (4 channels x 432 sites, forced-distributed
# one-rank RCCL group): per-channel streams vs staggered channels, ABAB
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4st}
: > gpurun_out/ab_stagger_$T.jsonl
for r in 1 2; do
  for mode in per-channel staggered; do
    TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
      timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 --warmup 3 \
      --no-extras --cpu-sample 0 --channel-streams $mode > gpurun_out/d.tmp 2> gpurun_out/dist432_${mode}_$T.err || exit $?
    tail -1 gpurun_out/d.tmp >> gpurun_out/ab_stagger_$T.jsonl
    python3 -c "import json; d=json.loads(open('gpurun_out/d.tmp').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['check_vs_oracle'])"
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multichannel.py > gpurun_out/mc_$T.log 2>&1 || exit $?
grep -E "passed|failed" gpurun_out/mc_$T.log | tail -1
echo $T-ok
