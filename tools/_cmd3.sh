set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/mb/mb_stats 1024 3 > gpurun_out/mb_r1s2c.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1s2c.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r1s2c.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r1s2c.log
for c in 0 1 2 3; do
  TMH_FUSED_CFG=$c timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --pipeline fused > gpurun_out/bench_cfg$c.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_cfg$c.json').read().strip().splitlines()[-1]); print('cfg$c', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
