#!/bin/bash
# PMC passes over the C5 GEMM kernels (tools/prof_gemm.py), one pass per run.
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/pmcg/pass$i -o run --output-format csv -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pmcg/pass$i.log 2>&1
done
echo done
