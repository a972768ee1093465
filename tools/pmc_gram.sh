set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/pmc_gram
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/pass$i -o run --output-format csv -- python3 $R/tools/prof_gram.py 3 > $O/pass$i.log 2>&1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/tools/prof_gram.py 10 > $O/stats.log 2>&1
echo done
