#!/bin/bash
# PMC passes over the bench's C5 line (x3 pre-split GEMMs); one counter group per run
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/pmc_c5
mkdir -p $O
ARGS="--no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 2 --warmup 1 --c5-steps 3 --c5-warmup 1"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $O/pass$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/pass$i.log 2>&1
done
echo done
