set -u
bash tools/gpu_check.sh r1s2a; rc=$?
tail -5 gpurun_out/gpu_tests_r1s2a.log; cat gpurun_out/smoke_r1s2a.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
STEPS=3 bash tools/gpu_ab.sh "sep||--pipeline separate" "fused||--pipeline fused"
