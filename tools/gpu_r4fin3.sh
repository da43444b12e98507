#!/bin/bash
# r4fin3: the final tree (with the rare lists) on one box -- build from source,
# GPU suite + smoke, default bench line, bright bench, kernel-trace stats for
# standard and bright
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4fin3}
bash tools/gpu_r4fin.sh $T || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --distribution bright > gpurun_out/bench_bright_$T.json 2> gpurun_out/bench_bright_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_bright_$T.json')); print('bright', d['value'], d['check_vs_oracle'])"
for dist in synthetic bright; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_${dist}_$T -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras --distribution $dist > gpurun_out/rocprof_${dist}_$T.log 2>&1 || exit $?
done
echo $T-all-ok
