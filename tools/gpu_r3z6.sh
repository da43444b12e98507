#!/bin/bash
# r3z6: chain pass staging: 1,024 threads with two barriers per site vs 960 / 896 threads with a double-buffered stage
mkdir -p gpurun_out
timeout -k 10 500 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3z6.txt 2>&1 || exit $?
