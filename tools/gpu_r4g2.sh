#!/bin/bash
# r4g2: final inflate build: GPU suite + smoke, inflate bench, input-path
# stream, run_job with GPU decode on a 1,536-site job
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4g2}
bash tools/gpu_build.sh $T || exit $?
bash tools/gpu_check.sh $T
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -1
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_inflate.py --distinct 16 --block 128 --reps 3 --lanes 4,8,16 > gpurun_out/bench_inflate_$T.json 2> gpurun_out/bench_inflate_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_inflate_$T.json')); print(d['gpu_kernel_ms_per_block'], d['inflate_kernels_sites_per_s'], d['gpu_equals_host'], {k: v['kernel_ms']['inflate'] for k, v in d['lanes_sweep'].items()})"
timeout -k 10 500 python tools/bench_input_path.py --blocks 128,256 > gpurun_out/input_path_$T.jsonl 2> gpurun_out/input_path_$T.err || exit $?
python3 -c "import json; [print(json.loads(l)['block'], json.loads(l)['gpu_inflate_stream_sites_per_s'], json.loads(l)['gpu_equals_host']) for l in open('gpurun_out/input_path_$T.jsonl')]"
timeout -k 10 900 python tools/bench_input.py --sites 128 --threads 16 --repeat 12 --device-block 128 > gpurun_out/bench_input_$T.json 2> gpurun_out/bench_input_$T.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_input_$T.json')); print({k: v for k, v in d.items() if 'run_job' in k or 'same' in k})"
echo $T-ok
