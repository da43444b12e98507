#!/bin/bash
# r4fin: the final round-4 tree on one box -- build from source, the full GPU
# suite + smoke, then the default bench line (extras and CPU baseline included)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4fin}
bash tools/gpu_build.sh $T || exit $?
bash tools/gpu_check.sh $T
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -2
tail -2 gpurun_out/smoke_$T.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$T.json')); x=d['extras']; print(d['value'], d['check_vs_oracle'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), x.get('one_job_at_a_time'), {k: v for k, v in x.get('input_path',{}).items() if 'per_s' in k})"
echo $T-ok
