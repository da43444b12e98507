#!/bin/bash
# r4x: round-4 evidence on one box: build, full GPU suite + smoke, headline
# bench (one full run with extras and CPU baseline, then repeats), bright,
# kernel-trace stats and HBM traffic (FETCH_SIZE / WRITE_SIZE in separate
# passes) for standard and bright, the N = 8 shard-size layout
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4x}
bash tools/gpu_build.sh $T || exit $?
bash tools/gpu_check.sh $T
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$T.json')); print(d['value'], d['check_vs_oracle'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d['extras'].get('one_job_at_a_time'), d['extras'].get('input_path',{}).get('gpu_inflate_stream_sites_per_s'))"
: > gpurun_out/bench_repeat_$T.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras > gpurun_out/b.tmp 2>> gpurun_out/bench_repeat_$T.err || exit $?
  cat gpurun_out/b.tmp >> gpurun_out/bench_repeat_$T.jsonl
done
python3 -c "import json; v=[json.loads(l)['value'] for l in open('gpurun_out/bench_repeat_$T.jsonl')]; print('repeats', v)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --distribution bright > gpurun_out/bench_bright_$T.json 2> gpurun_out/bench_bright_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_bright_$T.json')); print('bright', d['value'], d['check_vs_oracle'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_$T -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras > gpurun_out/rocprof_$T.log 2>&1 || exit $?
for dist in synthetic bright; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${dist}_$T -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-extras --no-profile --distribution $dist > gpurun_out/pmc_fetch_${dist}_$T.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${dist}_$T -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-extras --no-profile --distribution $dist > gpurun_out/pmc_write_${dist}_$T.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_${dist}_$T gpurun_out/pmc_write_${dist}_$T --sites 3456 --height 2160 --width 2560 -o gpurun_out/pmc_traffic_${dist}_$T.json || exit $?
done
TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
  timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 --warmup 3 \
  --no-extras --cpu-sample 0 > gpurun_out/dist432_$T.json 2> gpurun_out/dist432_$T.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/dist432_$T.json').read().strip().splitlines()[-1]); print('dist432', d['value'], d['ms_per_step'], d['check_vs_oracle'])"
echo $T-ok
