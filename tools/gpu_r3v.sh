#!/bin/bash
# r3v: two-plane smoothing (tmh_smooth2_f64_device): GPU parity suite, then
# three headline bench runs (smooth kernel time per job from the bench JSON)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r3v.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_r3v_$i.json 2> gpurun_out/bench_r3v_$i.err || exit $?
done
