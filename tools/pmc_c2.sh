#!/bin/bash
# PMC passes over the C2 staged kernel (tools/prof_c2.py), one rocprofv3 run per pass
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
mkdir -p $R/gpurun_out/pmc_c2
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_c2/avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/pmc_c2/pass$i -o run --output-format csv -- python3 $R/tools/prof_c2.py 3 > $R/gpurun_out/pmc_c2/pass$i.log 2>&1
done
echo done
