#!/bin/bash
# r3e: fold tail microbenchmark (dense vs production fold vs fold2 variants)
mkdir -p gpurun_out
timeout -k 10 240 ./tools/mb/mb_fold 3456 5 0 > gpurun_out/mb_fold_r3f.txt 2>&1 || exit $?
timeout -k 10 240 ./tools/mb/mb_fold 3456 3 1 > gpurun_out/mb_fold_bright_r3f.txt 2>&1 || exit $?
for i in 1 2; do
  for b in 0 64; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras --block-sites $b > gpurun_out/bench_blk${b}_r3f_$i.json 2> gpurun_out/bench_blk${b}_r3f_$i.err || exit $?
  done
done
