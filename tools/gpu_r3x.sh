#!/bin/bash
# r3x: chain pass variants (prefetch of the next site, site-part counts)
mkdir -p gpurun_out
timeout -k 10 400 tools/mb/mb_chain 3456 3 > gpurun_out/mb_chain_r3x.txt 2>&1 || exit $?
