# VALU / SALU / LDS instruction mix and issue counters of one Sankoff entry
# point at C4 size (tools/prof_kernels.py), one rocprofv3 --pmc pass each.
#   bash tools/pmc_mix.sh [fused|fwd|bwd] [trees]
set -e
R=$GRAFT_REPO_ROOT
W=${1:-fused}
T=${2:-128}
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/pmc_mix_$W
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU2 SQ_INSTS_VMEM_RD"
P3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P4="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/pass$i -o run --output-format csv -- python3 $R/tools/prof_kernels.py --which $W --iters 3 --trees $T > $O/pass$i.log 2>&1
done
echo done
