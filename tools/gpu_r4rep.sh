#!/bin/bash
# r4rep: the final tree -- five more default-config bench processes, and the
# N = 8 shard-size layout (4 x 432 sites, forced-distributed one-rank group)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4rep}
: > gpurun_out/bench_repeat_$T.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/b.tmp 2>> gpurun_out/bench_repeat_$T.err || exit $?
  cat gpurun_out/b.tmp >> gpurun_out/bench_repeat_$T.jsonl
done
python3 -c "import json; v=[json.loads(l)['value'] for l in open('gpurun_out/bench_repeat_$T.jsonl')]; print('repeats', v)"
TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
  timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 --warmup 3 \
  --no-extras --cpu-sample 0 > gpurun_out/dist432_$T.json 2> gpurun_out/dist432_$T.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/dist432_$T.json').read().strip().splitlines()[-1]); print('dist432', d['value'], d['ms_per_step'])"
echo $T-ok
