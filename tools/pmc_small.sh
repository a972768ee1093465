#!/bin/bash
# PMC passes (one rocprofv3 run each) over tools/prof_small.py:
#   tools/pmc_small.sh C3  -> gpurun_out/pmc_C3/pass*/run_counter_collection.csv
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/pmc_$1
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P -d $O/pass$i -o run --output-format csv -- python3 $R/tools/prof_small.py $1 3 > $O/pass$i.log 2>&1
done
echo done
