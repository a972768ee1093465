#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only; gfx950 slots):
# usage: tools/pmc_passes.sh OUTDIR [prof_kernels args]
set -e
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P -d "$OUT/pass$i" -o run --output-format csv -- python3 "$ROOT/tools/prof_kernels.py" "$@" > "$OUT/pass$i.log" 2>&1
done
