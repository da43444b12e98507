#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 ./tools/mb/mb_welford 3456 3 0 > gpurun_out/mb_welford_r3h.txt 2>&1 || exit $?
bash tools/ab_multi.sh wf_r3h 3 build_ab/wf_old/libtmhip.so build_ab/wf_new/libtmhip.so
