#!/bin/bash
# r4rl: fused pass, rare histogram values (beyond the LDS slice) by a loop over
# each lane's rare halves instead of eight masked sections: the full GPU suite
# with the new library, then bench ABAB against the previous build (ab_base/)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r4rl}
bash tools/gpu_check.sh $T
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/ab_fused_rareloop_$T.jsonl
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab_base/libtmhip.so; else L=$PWD/tmlibrary_amd/hip/libtmhip.so; fi
    for dist in bright synthetic; do
      TMH_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --distribution $dist --jobs-in-flight 1 > gpurun_out/b.tmp 2>> gpurun_out/ab_fused_rareloop_$T.err || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/b.tmp')); d['ab']={'lib': '$lib', 'jobs': 1}; print(json.dumps(d))" >> gpurun_out/ab_fused_rareloop_$T.jsonl
      python3 -c "import json; d=json.load(open('gpurun_out/b.tmp')); k=d['kernels']; print('$lib $dist', d['value'], d['check_vs_oracle'], k['welford']['avg_ms'], k['correct_hist']['avg_ms'])"
    done
  done
done
echo $T-ok
