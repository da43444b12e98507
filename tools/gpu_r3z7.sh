#!/bin/bash
# r3z7: chain pass staging of the seam lines only (one barrier per site) vs the whole workgroup
mkdir -p gpurun_out
timeout -k 10 500 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3z7.txt 2>&1 || exit $?
