#!/bin/bash
# SQ counters of the inflate kernels (three passes, each its own run)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d gpurun_out/zpmc_$1_p$i -o run --output-format csv -- python3 tools/inflate_prof.py --block 128 --lanes 8 --distinct 4 > gpurun_out/zpmc_$1_p$i.log 2>&1 || exit $?
done
echo zpmc-ok
