#!/bin/bash
# MFMA-busy / issue counters of the C5 GEMM kernels, v3 (TREX_GRAM=3,
# TREX_MF=3) against v5 (default), one --pmc pass per run.
#   bash tools/pmc_gemm_ab.sh  (on the GPU box) -> gpurun_out/pmcab/{v3,v5}/pass*/
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
for v in 3 5; do
  i=0
  for P in "$P1" "$P2" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    mkdir -p $R/gpurun_out/pmcab/v$v
    TREX_GRAM=$v TREX_MF=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/pmcab/v$v/pass$i -o run --output-format csv -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pmcab/v$v/pass$i.log 2>&1
  done
  for k in "gram_kernel3" "gram_kernel5<13, true" "gram_kernel5<13, false" "gram_kernel2<false" \
           "mf_kernel3<5, false" "mf_kernel5<5, false, true" "mf_kernel5<5, false, false" "mf_kernel2<false"; do
    echo "== v$v $k" >> $R/gpurun_out/pmcab/summary.txt
    python3 $R/tools/pmc_sum.py $R/gpurun_out/pmcab/v$v "$k" >> $R/gpurun_out/pmcab/summary.txt
  done
done
echo done
