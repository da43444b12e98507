#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${1:-diag}
timeout -k 10 300 python tools/diag_pct.py > gpurun_out/diag_$TAG.log 2>&1
rc=$?
echo "diag rc=$rc" >> gpurun_out/diag_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_check.sh $TAG
