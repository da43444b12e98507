#!/bin/bash
# GPU-box check: parity tests, then smoke.  Each GPU step has its own time
# limit; a crash/abort/timeout (rc not 0/1) ends the script there.
set -u
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -ra --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1
rc2=$?
echo "smoke rc=$rc2" >> gpurun_out/smoke_$TAG.log
exit $rc
