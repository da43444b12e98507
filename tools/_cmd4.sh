set -u
mkdir -p gpurun_out
MB_WF=1 timeout -k 10 300 tools/mb/mb_stats 1024 3 > gpurun_out/mb_r1s2d.txt 2>&1 || exit $?
